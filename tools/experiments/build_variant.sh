# Build a measurement variant of the in-tree library into opendht_amd/ab/<name>.so: copies csrc to a
# temp dir, applies a python edit script (which edits batch.hip in its cwd), builds there.  The
# production sources are never changed (the Makefile takes no extra defines: measurement switches
# are source edits, kept out of the shipped library).   usage: bash tools/experiments/build_variant.sh edit.py name
set -e
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
ED=$(cd "$(dirname "$1")" && pwd)/$(basename "$1")
T=$(mktemp -d /tmp/dhtgpu_var.XXXXXX)
mkdir -p "$T/opendht_amd" "$T/include"
cp -r "$ROOT/opendht_amd/csrc" "$T/opendht_amd/" && rm -rf "$T/opendht_amd/csrc/build" "$T/opendht_amd/csrc/build_ab"
cp -r "$ROOT/include/." "$T/include/"
(cd "$T/opendht_amd/csrc" && python3 "$ED")
make -C "$T/opendht_amd/csrc" -j8 >/dev/null
mkdir -p "$ROOT/opendht_amd/ab"
cp "$T/opendht_amd/libdhtgpu.so" "$ROOT/opendht_amd/ab/$2.so"
rm -rf "$T"
echo "variant $1 -> opendht_amd/ab/$2.so"
