#!/bin/bash
# serial-stream kernel traces of the ResNet-50 bench, folded BN vs not (TDL_BN_CONV_FOLD)
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out
TDL_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_fold -o run -- python3 $R/bench.py --steps 5 --warmup 3 > $R/gpurun_out/prof_fold.log 2>&1 || exit $?
TDL_BN_CONV_FOLD=0 TDL_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_nofold -o run -- python3 $R/bench.py --steps 5 --warmup 3 > $R/gpurun_out/prof_nofold.log 2>&1
