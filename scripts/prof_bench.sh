# rocprofv3 kernel trace + stats of a short bench run: bash scripts/prof_bench.sh NAME [bench args]
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
N=$1; shift
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$N -o run -- python3 $R/bench.py --steps 5 --warmup 3 "$@" > $R/gpurun_out/prof_$N.log 2>&1
