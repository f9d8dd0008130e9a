# in-step A/B of the BN backward reduce grid (bench.py, ResNet-50 b256)
set -u
for v in "base:" "b1024:TDL_BN_RED_BLOCKS=1024" "b2048m4:TDL_BN_RED_BLOCKS=2048 TDL_BN_RED_MINR=4" "b1024m8:TDL_BN_RED_BLOCKS=1024 TDL_BN_RED_MINR=8" "base2:" "b256:TDL_BN_RED_BLOCKS=256"; do
  tag=${v%%:*}; envs=${v#*:}
  echo -n "$tag " >> gpurun_out/red_ab.log
  env $envs timeout -k 10 120 python bench.py --steps 40 --warmup 5 2>/dev/null | grep -o '"value": [0-9.]*' >> gpurun_out/red_ab.log || exit $?
done
