set -o pipefail
STEPS="ab" ARMS="main ab/nw8.so ab/nw16.so main ab/nw8.so ab/nw16.so" bash scripts/r05_iter.sh
