#!/bin/bash
# re-check decided switches on the current tree: each pair alternated twice on the same box
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
for spec in ${SPECS:-"z_gemm:2 1" "gemm_proj:1 0" "gemm_proj_dgrad:1 0" "pw_z_wide:1 0" "wgrad_deep:1 0"}; do
  name=${spec%%:*}; vals=${spec#*:}
  AB_ENV=$name AB_VALUES="$vals" TAG=rc_$name bash tools/gpu/ab_env.sh || exit 1
done
