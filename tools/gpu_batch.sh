export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r03f; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_select.py -x -q --timeout 120 --timeout-method thread > $O/select.log 2>&1 || { tail -20 $O/select.log; exit 1; }
tail -2 $O/select.log
timeout -k 10 300 bash tools/hbm_roofline.sh $O/hbm > $O/hbm.log 2>&1 || exit 1
grep select $O/hbm/hbm_roofline.txt
for fam in default wide; do
  if [ $fam = default ]; then E=""; else E="DD_CONV_TILE=wide"; fi
  env $E timeout -k 10 200 python -u tools/conv_micro.py --only conv --batch 1024 --iters 10 --shapes 64:64:32,128:64:32,256:64:32,64:128:32,128:128:16,256:128:16 > $O/d1_$fam.txt 2>&1 || exit 1
  grep TF $O/d1_$fam.txt
done
bash tools/gpu_round.sh r03f tests smoke bench || exit 1
