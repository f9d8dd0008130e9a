cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/bnmicro -o run -- python3 $R/tools/bn_micro.py > $R/gpurun_out/bnmicro.log 2>&1
