set -o pipefail
bash scripts/r05_cmd14.sh && bash scripts/r05_prof.sh
