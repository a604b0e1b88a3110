set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_reference_testdata.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/reftd.log 2>&1 || { tail -30 gpurun_out/reftd.log; exit 1; }
tail -2 gpurun_out/reftd.log
timeout -k 10 300 python tools/bench_c3.py > gpurun_out/c3.log 2>&1 || { tail -30 gpurun_out/c3.log; exit 1; }
cat gpurun_out/c3.log
for c in noise gradient blobs; do BATCH=1 CONTENT=$c WEBPGPU_LIB=webp_amd/libwebpgpu_stamps.so timeout -k 10 120 python tools/debug_enc_phases.py; done > gpurun_out/ph1.log 2>&1
cat gpurun_out/ph1.log
