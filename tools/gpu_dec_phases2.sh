mkdir -p gpurun_out; export TMPDIR=/tmp
WEBPGPU_LIB=webp_amd/libwebpgpu_stamps.so timeout -k 10 200 python tools/debug_split_phases.py > gpurun_out/sp.log 2>&1 || { tail -20 gpurun_out/sp.log; exit 1; }
grep p_i4 gpurun_out/sp.log
WEBPGPU_LIB=webp_amd/libwebpgpu_stamps.so SIZE=1080 BATCH=64 timeout -k 10 200 python tools/debug_split_phases.py > gpurun_out/sp2.log 2>&1 || { tail -20 gpurun_out/sp2.log; exit 1; }
grep p_i4 gpurun_out/sp2.log
for k in bands split; do WG_DECODE_KERNEL=$k timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_$k.log 2>&1 || { tail -20 gpurun_out/bench_$k.log; exit 1; }; python3 -c "
import json,sys; d=json.loads(open('gpurun_out/bench_$k.log').read().strip().splitlines()[-1]); print('$k', d['value'], d['stage_ms_isolated'])"; done
