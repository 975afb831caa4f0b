# Build the working tree's libdhtgpu with extra compile flags into opendht_amd/ab/<name>.so
# (measurement variants for A/B runs).   usage: bash tools/experiments/build_variant.sh <name> "<flags>"
set -e
NAME=$1; FLAGS=$2
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
T=$(mktemp -d /tmp/dhtgpu_var.XXXXXX)
mkdir -p $T/opendht_amd $T/include
cp -r "$ROOT/opendht_amd/csrc" $T/opendht_amd/ && rm -rf $T/opendht_amd/csrc/build $T/opendht_amd/csrc/build_ab
cp "$ROOT"/include/*.h $T/include/
make -C $T/opendht_amd/csrc -j8 EXTRA="$FLAGS" >/dev/null
mkdir -p "$ROOT/opendht_amd/ab"
cp $T/opendht_amd/libdhtgpu.so "$ROOT/opendht_amd/ab/$NAME.so"
rm -rf $T
echo "built $NAME ($FLAGS)"
