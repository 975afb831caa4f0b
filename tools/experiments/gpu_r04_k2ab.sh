# K2 variants only (no tests, no PMC): name=path pairs three times each.  usage: bash tools/experiments/gpu_r04_k2ab.sh tag name=path...
set -o pipefail
TAG=$1; shift
bash tools/experiments/gpu_k2_libs.sh $TAG "$@"
