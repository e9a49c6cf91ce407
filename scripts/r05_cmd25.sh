set -o pipefail
bash scripts/profile_r05.sh ingest || exit 1
python3 scripts/summarize_profile.py gpurun_out/prof_ingest r05 || exit 1
mkdir -p gpurun_out/r05_profiles && cp profiles/r05/kernel_stats.csv profiles/r05/pmc_summary.json profiles/r05/summary.md gpurun_out/r05_profiles/
