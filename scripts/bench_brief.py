"""One line per bench JSON file: value, ms/step and the per-kernel breakdown."""
import json
import os
import sys

for f in sys.argv[1:]:
    if not os.path.exists(f):
        continue
    d = json.load(open(f))
    print(f, round(d["value"] / 1e9, 2), "G updates/s", round(d["ms_per_step"], 3), "ms/step",
          d.get("breakdown_ms_per_step"))
