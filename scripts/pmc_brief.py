"""Per-kernel averages of a rocprofv3 --pmc counter_collection.csv (cms:: kernels):
counters summed per dispatch, averaged over dispatches; VGPR/LDS per kernel."""
import collections
import csv
import glob
import sys

for d in sys.argv[1:]:
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
    if not f:
        continue
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    info = {}
    for r in csv.DictReader(open(f[0])):
        n = r["Kernel_Name"]
        if not n.startswith("cms::"):
            continue
        n = n.split("(")[0]
        per[n][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[n].add(r["Dispatch_Id"])
        info[n] = (r["VGPR_Count"], r["Accum_VGPR_Count"], r["SGPR_Count"], r["LDS_Block_Size"], r["Workgroup_Size"])
    print("==", d)
    for n, c in per.items():
        k = len(disp[n])
        v = " ".join(f"{cn}={cv / k:.4g}" for cn, cv in sorted(c.items()))
        print(f"{n} [vgpr {info[n][0]}+{info[n][1]} sgpr {info[n][2]} lds {info[n][3]} wg {info[n][4]}] {v}")
