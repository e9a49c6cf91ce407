set -o pipefail
STEPS="ab" ARMS="main ab/nw2.so ab/nw1.so main ab/nw2.so ab/nw1.so" bash scripts/r05_iter.sh
