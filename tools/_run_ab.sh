cd $GRAFT_REPO_ROOT && BENCH_ARGS="--no-walk10m" LIBS="w7 prev main w7 prev main w6 w7" bash tools/gpu_ablib.sh
