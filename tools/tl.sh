mkdir -p gpurun_out && timeout -k 10 400 python -m pytest tests/test_gpu_lsd.py -x -q > gpurun_out/spec_tests.log 2>&1; rc=$?; tail -3 gpurun_out/spec_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/time_lsd.py 256 || exit 1
for b in 1024 1536; do timeout -k 10 200 python tools/time_lsd.py $b | head -1 || exit 1; done
