set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
PBL_LIB=exp/snapst.so timeout -k 10 300 python scripts/snap_stamps.py 16384
