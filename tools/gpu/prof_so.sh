#!/bin/bash
# rocprofv3 kernel stats of the eager step with the in-tree .so and with RT1_HIP_SO=$BASE_SO (same box)
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
TAG=${TAG:-pso}
PROF_TAG=prof_${TAG}1 PROF_STEPS=3 PROF_TOP=40 bash tools/gpu/prof.sh > /dev/null && \
RT1_HIP_SO=$BASE_SO PROF_TAG=prof_${TAG}0 PROF_STEPS=3 PROF_TOP=40 bash tools/gpu/prof.sh > /dev/null && echo done
