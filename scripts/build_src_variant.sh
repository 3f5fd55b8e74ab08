# Fast variant build: one source of pebble_amd/csrc with extra hipcc flags,
# linked with the other sources' release objects (pebble_amd/.obj) -> exp/<name>.so.
# Usage: bash scripts/build_src_variant.sh <source.hip> <name> [extra hipcc flags]
set -e
src=$1; name=$2; shift 2
root=$(git rev-parse --show-toplevel)
mkdir -p "$root/exp"
cd "$root/pebble_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -pthread "$@" -c "$src" -o "/tmp/$name.o"
others=$(ls "$root"/pebble_amd/.obj/*.rel.o | grep -v "/${src%.hip}.rel.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -pthread "/tmp/$name.o" $others -o "$root/exp/$name.so"
echo "$root/exp/$name.so"
