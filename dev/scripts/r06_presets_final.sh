# Final preset numbers: Xception-41 b128, DeepLab preset b32 (graph), ResNet-152 fp8 vs bf16 b512 (graph)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
p() { tag=$1; shift; timeout -k 10 400 python bench.py "$@" > gpurun_out/r06_pf.log 2>&1 || exit 1; echo "## $tag"; tail -1 gpurun_out/r06_pf.log; }
p "xception41 b128" --model xception41 --batch 128 --image-size 299
p "deeplab preset b32 graph" --model deeplab_ref --batch 32 --graph
p "resnet152 fp8 b512 graph" --model resnet152 --batch 512 --fp8 --graph --steps 10 --warmup 3
p "resnet152 bf16 b512 graph" --model resnet152 --batch 512 --graph --steps 10 --warmup 3
