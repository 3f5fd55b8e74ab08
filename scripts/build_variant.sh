# Build libpebble_amd.so from a git revision into exp/<name>.so (for scripts/ab.sh).
# Usage: bash scripts/build_variant.sh <rev|.> <name> [extra hipcc flags]   (. = the working tree)
set -e
rev=$1; name=$2; shift 2
root=$(git rev-parse --show-toplevel)
wt=$(mktemp -d /tmp/pbl_wt.XXXX)
if [ "$rev" = "." ]; then cp -r "$root/pebble_amd" "$root/include" "$wt/"; else git -C "$root" worktree add -q --detach "$wt" "$rev"; fi
mkdir -p "$root/exp"
(cd "$wt/pebble_amd/csrc" && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -pthread "$@" \
  $(ls *.hip) $(ls *.cpp) \
  -o "$root/exp/$name.so")
if [ "$rev" = "." ]; then rm -rf "$wt"; else git -C "$root" worktree remove --force "$wt"; fi
echo "$root/exp/$name.so"
