#!/bin/bash
# block 1's residual gradient in the unified depthwise backward's store (RT1_DW_RES): tests + same-box bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out; export TMPDIR=/tmp
TESTS="tests/test_backbone_gpu.py tests/test_parity_gpu.py" AB_ENV=RT1_DW_RES TAG=dwres bash tools/gpu/ab_env.sh
