# BN kernel knob sweep (dev/tools/bn_micro.py, one process per setting)
set -u
for v in "base:" "minr4:TDL_BN_RED_MINR=4" "minr8:TDL_BN_RED_MINR=8" "minr4u8:TDL_BN_RED_MINR=8 TDL_BN_RED_U=8" "minr4b1024:TDL_BN_RED_MINR=4 TDL_BN_RED_BLOCKS=1024" "ewu2:TDL_BN_BWD_U=2 TDL_BN_APPLY_U=2" "ewu2b1024:TDL_BN_BWD_U=2 TDL_BN_APPLY_U=2 TDL_BN_EW_BLOCKS=1024" "ewu4b1024:TDL_BN_BWD_U=4 TDL_BN_APPLY_U=4 TDL_BN_EW_BLOCKS=1024" "ewb4096:TDL_BN_EW_BLOCKS=4096" "ewu2b4096:TDL_BN_BWD_U=2 TDL_BN_APPLY_U=2 TDL_BN_EW_BLOCKS=4096"; do
  tag=${v%%:*}; envs=${v#*:}
  env $envs BN_TAG=$tag timeout -k 10 120 python dev/tools/bn_micro.py >> gpurun_out/bn_micro2.log 2>&1 || exit $?
done
