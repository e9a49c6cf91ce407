import csv,sys
rows=list(csv.DictReader(open("gpurun_out/kt/run_kernel_trace.csv")))
rows.sort(key=lambda r:int(r["Start_Timestamp"]))
idx=[i for i,r in enumerate(rows) if "k_p1_hist" in r["Kernel_Name"]]
for a,b in zip(idx[3:5], idx[4:6]):
    seg=rows[a:b]
    t0=int(seg[0]["Start_Timestamp"]); t1=int(seg[-1]["End_Timestamp"])
    busy=sum(int(r["End_Timestamp"])-int(r["Start_Timestamp"]) for r in seg)
    print("span %.1f busy %.1f next %.1f" % ((t1-t0)/1e3, busy/1e3, (int(rows[b]["Start_Timestamp"])-t1)/1e3))
    prev=None
    for r in seg:
        s=int(r["Start_Timestamp"]); e=int(r["End_Timestamp"])
        if prev and s-prev>2000: print("  gap %.1f before %s" % ((s-prev)/1e3, r["Kernel_Name"][:40]))
        prev=e
