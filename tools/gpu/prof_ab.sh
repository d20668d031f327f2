#!/bin/bash
# rocprofv3 kernel stats of the eager step with $AB_ENV=0 and =1 (same box) -> gpurun_out/prof_${TAG}{0,1}
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
TAG=${TAG:-pab}
env $AB_ENV=1 PROF_TAG=prof_${TAG}1 PROF_STEPS=3 PROF_TOP=40 bash tools/gpu/prof.sh > /dev/null && \
env $AB_ENV=0 PROF_TAG=prof_${TAG}0 PROF_STEPS=3 PROF_TOP=40 bash tools/gpu/prof.sh > /dev/null && echo done
