set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/fb2; mkdir -p $O
LIB=ablate_libs/libnicnes_blkchk.so timeout -k 10 400 python -u scripts/dev/debug_sample_fb.py 512 2>&1 | head -c 20000000 > $O/fb_chk.log
timeout -k 10 400 python -u scripts/dev/debug_sample_fb.py 512 > $O/fb.log 2>&1
echo ok
