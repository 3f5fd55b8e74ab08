# Fast variant build: rowblk_decode.hip with extra hipcc flags, linked with the
# other sources' release objects (pebble_amd/.obj) -> exp/<name>.so.
# Usage: bash scripts/build_row_variant.sh <name> [extra hipcc flags]
set -e
name=$1; shift
root=$(git rev-parse --show-toplevel)
mkdir -p "$root/exp"
cd "$root/pebble_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -pthread "$@" -c rowblk_decode.hip -o "/tmp/$name.o"
others=$(ls "$root"/pebble_amd/.obj/*.rel.o | grep -v rowblk_decode)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -pthread "/tmp/$name.o" $others -o "$root/exp/$name.so"
echo "$root/exp/$name.so"
