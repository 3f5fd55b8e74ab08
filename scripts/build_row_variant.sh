# Fast variant build: one source (rowblk_decode.hip, or $SRC) with extra hipcc
# flags, linked with the other sources' release objects (pebble_amd/.obj) ->
# exp/<name>.so, loaded through PBL_LIB=exp/<name>.so.
# Usage: [SRC=zstd.hip] bash scripts/build_row_variant.sh <name> [extra hipcc flags]
set -e
name=$1; shift
src=${SRC:-rowblk_decode.hip}
root=$(git rev-parse --show-toplevel)
mkdir -p "$root/exp"
cd "$root/pebble_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -pthread "$@" -c "$src" -o "/tmp/$name.o"
others=$(ls "$root"/pebble_amd/.obj/*.rel.o | grep -v "/${src%%.*}.rel.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -pthread "/tmp/$name.o" $others -o "$root/exp/$name.so"
echo "$root/exp/$name.so"
