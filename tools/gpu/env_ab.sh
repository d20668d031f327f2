#!/bin/bash
# Same-box A/B of one environment switch on the working tree's build: the GPU tests named in AB_TESTS first, then
# bench.py alternated AB_REPS times with AB_OFF / AB_ON (e.g. AB_OFF=RT1_DY_READY=0 AB_ON=RT1_DY_READY=1).
source "$(dirname "$0")/step.sh"
TAG=${AB_TAG:-env}
if [ -n "$AB_TESTS" ]; then
    run_step ${TAG}_tests 600 env $AB_ON python -u -m pytest -x -q --timeout 300 --timeout-method thread $AB_TESTS
fi
for rep in $(seq 1 ${AB_REPS:-2}); do
    TAIL=1 run_step ${TAG}_base_$rep 300 env $AB_OFF python -u bench.py --steps 20 --warmup 5
    TAIL=1 run_step ${TAG}_new_$rep 300 env $AB_ON python -u bench.py --steps 20 --warmup 5
done
