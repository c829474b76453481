#!/bin/bash
# Round-5 GPU call: the named GPU test files (one pytest process), then the profile set of the final sources
# (scripts/profile_r03.sh: kernel-trace stats + 4 PMC passes at 512 / 128 / 64 members per GPU, and the sampled
# decode at 512), post-processed on this side by scripts/make_profiles.py.
# usage (on the GPU box): bash scripts/gpu_r05_prof.sh TAG ["tests/test_a.py ..." | none] [POPS] [sample|nosample]
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-r05p}
O=gpurun_out/$TAG
mkdir -p $O
if [ "${2:-none}" != none ]; then
  timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread $2 > $O/tests.log 2>&1
fi
if [ "${3:-none}" != none ]; then
  bash scripts/profile_r03.sh $TAG "$3"
fi
if [ "${4:-nosample}" = sample ]; then
  bash scripts/profile_r03.sh ${TAG}s "512" --fitness sample
fi
echo ok
