# end-of-round numbers of the non-headline presets (same box): Xception-41 b128, the reference
# DeepLab preset b32 eager and graph
set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out; : > gpurun_out/others.log
run() { timeout -k 10 400 python bench.py "$@" 2>/dev/null | tail -1 | grep -o '"value": [0-9.]*' | sed "s/^/$* /" >> gpurun_out/others.log; }
run --model xception41 --batch 128
run --model deeplab_ref --batch 32
run --model deeplab_ref --batch 32 --graph
