#!/bin/bash
# serial-stream kernel traces of the ResNet-50 bench, dgrad-as-forward on vs off (TDL_DGRAD_AS_FWD)
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out
TDL_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_on -o run -- python3 $R/bench.py --steps 5 --warmup 3 > $R/gpurun_out/prof_on.log 2>&1 || exit $?
TDL_DGRAD_AS_FWD=0 TDL_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_off -o run -- python3 $R/bench.py --steps 5 --warmup 3 > $R/gpurun_out/prof_off.log 2>&1 || exit $?
cd $R && timeout -k 10 200 python bench.py > gpurun_out/b_on.log 2>&1 && TDL_DGRAD_AS_FWD=0 timeout -k 10 200 python bench.py > gpurun_out/b_off.log 2>&1 && timeout -k 10 200 python bench.py > gpurun_out/b_on2.log 2>&1
