#!/bin/bash
# K13 stride-2 forward: K13 tests, then the A/B against the library forward at ResNet-50's shapes
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/conv_s2
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv3x3_gpu.py tests/test_models_gpu.py tests/test_conv_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 3; }
tail -2 $O/tests.log
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 3; }
tail -1 $O/bench.log | cut -c1-300
