# rocprofv3 hardware counters over a few ResNet-50 b256 training steps (one pass per counter group,
# each within the per-block slot limits; --kernel-trace only alongside --pmc).
#   bash dev/scripts/pmc_bench.sh [model] [batch] [image]
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
M=${1:-resnet50}; B=${2:-256}; I=${3:-224}
run() {
  tag=$1; shift
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc "$@" --output-format csv \
    -d $R/gpurun_out/pmc_${M}_$tag -o run -- python3 $R/bench.py --model $M --batch $B \
    --image-size $I --steps 2 --warmup 1 > $R/gpurun_out/pmc_${M}_$tag.log 2>&1
}
run sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT \
    SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE || exit $?
run fetch FETCH_SIZE GRBM_GUI_ACTIVE || exit $?
run write WRITE_SIZE TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE || exit $?
