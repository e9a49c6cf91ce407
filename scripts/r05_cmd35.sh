set -o pipefail
STEPS="ab" ARMS="main ab/mg4.so ab/mg16.so main ab/mg4.so ab/mg16.so" bash scripts/r05_iter.sh
