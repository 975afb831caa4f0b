# Build libdhtgpu at a commit (default HEAD) into opendht_amd/ab/<name>.so for A/B runs against
# the in-tree build (tools/experiments/gpu_ab_lib.sh, tools/experiments/gpu_ab_libs.sh).   usage: bash tools/experiments/build_prev.sh [rev] [name]
set -e
REV=${1:-HEAD}; NAME=${2:-prev}
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
WT=$(mktemp -d /tmp/dhtgpu_wt.XXXXXX)
git -C "$ROOT" worktree add -q "$WT" "$REV"
make -C "$WT/opendht_amd/csrc" -j8 >/dev/null
mkdir -p "$ROOT/opendht_amd/ab"
cp "$WT/opendht_amd/libdhtgpu.so" "$ROOT/opendht_amd/ab/$NAME.so"
git -C "$ROOT" worktree remove --force "$WT"
echo "built $REV -> opendht_amd/ab/$NAME.so"
