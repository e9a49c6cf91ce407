#!/bin/bash
# Round-6 rocprofv3 passes (one counter group per run, kernel trace only; no
# sys/runtime trace).  Usage: scripts/profile_r06.sh {ingest|config2|cosine}
#   ingest  -- the headline (config-3 shape) bench command: kernel stats,
#              FETCH_SIZE, WRITE_SIZE
#   ingest_sq -- the same command: kernel stats, then one pass of SQ wave /
#              LDS counters (what the build kernels wait on)
#   config2 -- the config-2 line alone (bench.py --no-headline): the same passes
#   cosine  -- the config-4 job (scripts/cos_job_probe.py): kernel stats, then
#              MFMA busy / waits, LDS, L2 hit, FETCH_SIZE passes
# Summaries: scripts/summarize_profile.py / summarize_cos_pmc.py -> profiles/r06.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
MODE=${1:-ingest}
OUT=gpurun_out/prof_$MODE
rm -rf $OUT
mkdir -p $OUT
case $MODE in
  ingest|ingest_sq) CMD="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras --no-config1 --no-config2 --no-cosine-1m" ;;
  config2) CMD="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras --no-config1 --no-headline" ;;
  cosine)  CMD="python3 scripts/cos_job_probe.py ${COS_ARGS:-1000000 500000000 8192 100}" ;;
  *) echo "mode?"; exit 2 ;;
esac
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $CMD \
    > $OUT/trace.log 2>&1 || { echo "trace failed"; exit 1; }
echo "trace ok"
if [ "$MODE" = ingest_sq ]; then
  timeout -k 10 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
      SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $OUT/sq -o run --output-format csv -- $CMD \
      > $OUT/sq.log 2>&1 || { echo "sq pass failed"; exit 1; }
  echo "sq pass ok"
elif [ "$MODE" = cosine ]; then
  i=0
  for grp in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
             "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES" \
             "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE"; do
    i=$((i+1))
    timeout -k 10 400 rocprofv3 --pmc $grp -d $OUT/p$i -o run --output-format csv -- $CMD \
        > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
    echo "pass $i ok"
  done
else
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 400 rocprofv3 --pmc $ctr -d $OUT/$(echo $ctr | cut -d_ -f1 | tr A-Z a-z) -o run --output-format csv -- $CMD \
        > $OUT/$ctr.log 2>&1 || { echo "$ctr failed"; exit 1; }
    echo "$ctr ok"
  done
fi
