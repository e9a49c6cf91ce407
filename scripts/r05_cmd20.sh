set -o pipefail
SKIP_COS_PROF=1 bash scripts/r05_final.sh || exit 1
bash scripts/profile_r05.sh ingest_sq || exit 1
mkdir -p gpurun_out/r05_sq && cp -r gpurun_out/prof_ingest_sq/sq gpurun_out/r05_sq/ 2>/dev/null; ls gpurun_out/prof_ingest_sq
