mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_frames.py -x -q -m gpu --timeout 120 --timeout-method thread -k "import or analysis or nrgba or ssim" > gpurun_out/t.log 2>&1 || { echo FAIL; tail -40 gpurun_out/t.log; exit 1; }
tail -2 gpurun_out/t.log
STREAM_ONLY=1 REPS=20 timeout -k 10 200 python tools/bench_stages.py
