#!/bin/bash
# Same-box A/B of two source trees (Python + extension), e.g. HEAD in a git worktree with its own in-tree build vs the
# working tree:  git worktree add build/base_tree HEAD && (cd build/base_tree && python -c "import build; build.build()")
#   BASE_TREE=build/base_tree TAG=x bash tools/gpu/ab_tree.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
ROOT=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-abtree}
val() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for rep in ${REPS:-1 2 3}; do
  (cd "$BASE_TREE" && timeout -k 10 300 python -u bench.py --steps ${STEPS:-20} --warmup 5) > gpurun_out/abtree_${TAG}_base_$rep.log 2>&1 || { echo "base failed"; tail -5 gpurun_out/abtree_${TAG}_base_$rep.log; exit 1; }
  echo "base rep$rep: $(val gpurun_out/abtree_${TAG}_base_$rep.log)"
  (cd "$ROOT" && timeout -k 10 300 python -u bench.py --steps ${STEPS:-20} --warmup 5) > gpurun_out/abtree_${TAG}_new_$rep.log 2>&1 || { echo "new failed"; tail -5 gpurun_out/abtree_${TAG}_new_$rep.log; exit 1; }
  echo "new  rep$rep: $(val gpurun_out/abtree_${TAG}_new_$rep.log)"
done
