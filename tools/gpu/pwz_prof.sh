cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
RT1_PW_BWD_Z=1 PROF_TAG=prof_pwz1 PROF_STEPS=3 PROF_TOP=40 bash tools/gpu/prof.sh > /dev/null && RT1_PW_BWD_Z=0 PROF_TAG=prof_pwz0 PROF_STEPS=3 PROF_TOP=40 bash tools/gpu/prof.sh > /dev/null && echo done
