# A/B ablations of the LDS-DMA conv kernel (interleaved in one process per shape)
R=$GRAFT_REPO_ROOT
for shp in 256,56,64,64,3,1,1 256,14,512,512,3,2,1 256,28,128,128,3,1,1 256,14,1024,256,1,1,0; do
  python3 $R/tools/conv_ablate.py --shape $shp || exit $?
done
