#!/bin/bash
# Round-5 profile passes for the bench's roofline fields: the headline ingest
# (kernel stats, FETCH_SIZE, WRITE_SIZE) and the config-4 cosine job (kernel
# stats, MFMA / wait, LDS, L2, FETCH), summarised into profiles/r05 on the box
# (where bench.py reads them) and copied to gpurun_out/r05_profiles.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/profile_r05.sh ingest || exit 1
python3 scripts/summarize_profile.py gpurun_out/prof_ingest r05 || exit 1
bash scripts/profile_r05.sh cosine || exit 1
python3 scripts/summarize_cos_pmc.py gpurun_out/prof_cosine r05 || exit 1
mkdir -p gpurun_out/r05_profiles
cp profiles/r05/* gpurun_out/r05_profiles/
ls gpurun_out/r05_profiles
