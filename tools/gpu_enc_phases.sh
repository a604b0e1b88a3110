set -e
export WEBPGPU_LIB=webp_amd/libwebpgpu_stamps.so
for c in noise gradient blobs mix; do CONTENT=$c timeout -k 10 240 python tools/debug_enc_phases.py; done
