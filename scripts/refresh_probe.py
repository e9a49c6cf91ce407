"""Config-5 refresh probe: the 1M-item table of configs 3+4, then incremental
batches and cms_top_k_refresh with every phase timed (level-2 scopes).

usage: python scripts/refresh_probe.py [batches_per_refresh ...]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("CMS_RF_DEBUG", "1")
from bench import config3_shard  # noqa: E402
from mahout_amd import SketchTable  # noqa: E402
from mahout_amd.synth import zipf_stream_torch  # noqa: E402

SCOPES = ["refresh_full", "refresh_job", "refresh_fold", "refresh_redo", "limb_prep", "topk_all_multi_rows",
          "topk_all_waves", "topk_all_waves_f4", "topk_all_waves_i8", "top_k", "cosine_mfma", "cosine_mfma_limbs",
          "cosine_mfma_multi"]


def main():
    plan = [int(a) for a in sys.argv[1:]] or [1, 4]
    n, d, w, k = 1_000_000, 5, 8192, 100
    dev = torch.device("cuda:0")
    t = SketchTable(n, depth=d, width=w, seed=42, device=0)
    items, users = config3_shard(n, 10_000_000, 500_000_000, 0, 1, dev)
    t.ingest_device_rows(items, users, None, int(items.numel()))
    t.finalize()
    del items, users
    torch.cuda.empty_cache()
    st = t.stats()
    print("multi", st["multi_limb_owners"], "fp4", st["fp4_owners"], flush=True)
    t0 = time.perf_counter()
    t.top_k_refresh(k)
    print(f"whole job (depth 2k) {time.perf_counter() - t0:.2f} s", flush=True)
    seed = 0
    for nbat in plan:
        for _ in range(nbat):
            it_, us = zipf_stream_torch(10_000_000, n, 1_250_000, seed=777_000 + seed, device=dev)
            seed += 1
            t.ingest_device_rows(it_.contiguous(), us.contiguous(), None, int(it_.numel()))
        t.finalize()
        t.set_timing(True, level=2)
        t.reset_timing()
        t0 = time.perf_counter()
        t.top_k_refresh(k)
        wall = time.perf_counter() - t0
        touched, redone, full = t.refresh_stats()
        print(f"{nbat} batches: refresh {wall:.2f} s touched {touched / n:.3f} redone {redone} whole {full} "
              f"topk_redo {t.stats()['topk_redo']} classes {t.refresh_classes()}")
        for s in SCOPES:
            ms, cnt = t.timing(s)
            if cnt:
                print(f"   {s:22s} {ms:10.1f} ms  x{cnt}")
        sys.stdout.flush()
        t.set_timing(False)
    t.close()


if __name__ == "__main__":
    main()
