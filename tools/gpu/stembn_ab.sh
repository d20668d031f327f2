#!/bin/bash
# stem BN backward in the stem weight-gradient kernel's staging (RT1_STEM_BN_BWD): tests + same-box bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out; export TMPDIR=/tmp
TESTS="tests/test_backbone_gpu.py tests/test_parity_gpu.py tests/test_distributed_gpu.py" AB_ENV=RT1_STEM_BN_BWD TAG=stembn bash tools/gpu/ab_env.sh
