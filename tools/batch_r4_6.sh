set -e
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread > gpurun_out/q6_pytest.log 2>&1
bash tools/abl_sweep.sh d1 c2 static:16:0:0 dyn:16:0:0 static:12:0:0 dyn:12:0:0 static:32:0:0 dyn:32:0:0 static:16:0:0 dyn:16:0:0 dyn:18:0:0 dyn:24:0:0
bash tools/abl_sweep.sh d1c3 c3 static:16:0:0 dyn:16:0:0 static:16:0:0 dyn:16:0:0
bash tools/abl_sweep.sh d1c4 c4 static:16:0:0 dyn:16:0:0 static:16:0:0 dyn:16:0:0
