#!/bin/bash
# Same-box A/B of the working tree's build against build/base (the HEAD commit's build): the GPU tests named in
# AB_TESTS first, then bench.py alternated AB_REPS times.   AB_TAG=x AB_TESTS="tests/a.py tests/b.py" bash tools/gpu/ab_base.sh
source "$(dirname "$0")/step.sh"
SO=_rt1_hip.cpython-310-x86_64-linux-gnu.so
TAG=${AB_TAG:-ab}
if [ -n "$AB_TESTS" ]; then
    run_step ${TAG}_tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread $AB_TESTS
fi
for rep in $(seq 1 ${AB_REPS:-2}); do
    RT1_HIP_SO=build/base/$SO TAIL=1 run_step ${TAG}_base_$rep 300 python -u bench.py --steps 20 --warmup 5
    TAIL=1 run_step ${TAG}_new_$rep 300 python -u bench.py --steps 20 --warmup 5
done
