X="python bench.py --model xception41 --batch 128 --image-size 299"
bash scripts/gpu_run.sh \
 "tr32:300:$X" \
 "tr16:300:TDL_DW_TR=16 $X" \
 "tr10:300:TDL_DW_TR=10 $X" \
 "tr7:300:TDL_DW_TR=7 $X" \
 "tr5:300:TDL_DW_TR=5 $X" \
 "tr32b:300:$X"
