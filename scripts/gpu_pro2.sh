set -u
OUT=gpurun_out; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py -k "prologue or three_passes" > $OUT/pro_tests.log 2>&1 || { tail -30 $OUT/pro_tests.log; exit 3; }
tail -n 1 $OUT/pro_tests.log
timeout -k 10 400 python bench/resnet_flag_ab.py --flag madnn.ops:_BN_PROLOGUE --batch 1536 --windows 6 --steps 4 --json-out $OUT/ab_bn_prologue2.json > $OUT/ab_bn_prologue2.log 2>&1 || { tail -20 $OUT/ab_bn_prologue2.log; exit 5; }
tail -n 1 $OUT/ab_bn_prologue2.log
PROF_ENV=MADNN_BN_PROLOGUE bash scripts/gpu_prof_ab.sh > /dev/null
