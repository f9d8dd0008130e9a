cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in bf16 fp8; do
  F=""; [ $v = fp8 ] && F="--fp8"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$v -o run -- python3 $R/bench.py --model resnet152 --batch 128 --steps 5 --warmup 3 $F > $R/gpurun_out/prof_$v.log 2>&1 || exit $?
done
