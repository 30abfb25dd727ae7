#!/bin/bash
# Round-3 GPU check: targeted tests, attention variants, YOLO stem, bench, control-plane hop bench.
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_detect.py tests/test_gpu_transformer.py -x -v \
  --timeout 120 --timeout-method thread \
  -k "admission or upsample or log_mel or resnet_pipeline or lanes or attention or stem or gemm_fp8" > gpurun_out/t_r3c.log 2>&1 || { tail -40 gpurun_out/t_r3c.log; exit 1; }
grep -cE "PASSED" gpurun_out/t_r3c.log
for v in 0 10 11 12 13; do
  echo -n "attn variant $v: "; AIKO_ATTN_VARIANT=$v timeout -k 10 60 python scripts/op_bench.py attn | grep attn: || exit 1
done
echo -n "stem fast: "; timeout -k 10 60 python scripts/yolo_stem_bench.py || exit 1
echo -n "stem old:  "; AIKO_STEM_FAST=0 timeout -k 10 60 python scripts/yolo_stem_bench.py || exit 1
timeout -k 10 300 python bench.py --steps 40 --warmup 8 > gpurun_out/bench_r3c.log 2>&1 || { tail -20 gpurun_out/bench_r3c.log; exit 1; }
tail -1 gpurun_out/bench_r3c.log
AIKO_STEM_U8=0 timeout -k 10 300 python bench.py --steps 40 --warmup 8 > gpurun_out/bench_r3c_nou8.log 2>&1 || { tail -20 gpurun_out/bench_r3c_nou8.log; exit 1; }
echo -n "no-u8-stem: "; tail -1 gpurun_out/bench_r3c_nou8.log
timeout -k 10 300 python -m aiko_services_amd.tools.hop_bench --replicas 7 --hop-batch 8 --seconds 8 > gpurun_out/hop_box8.json 2>gpurun_out/hop_box8.err || exit 1
timeout -k 10 300 python -m aiko_services_amd.tools.hop_bench --replicas 7 --hop-batch 1 --seconds 8 > gpurun_out/hop_box1.json 2>gpurun_out/hop_box1.err || exit 1
cut -c1-330 gpurun_out/hop_box8.json gpurun_out/hop_box1.json
for op in gemm_qkv gemm_fc1 gemm_fc2 gemm_out; do
  for t in 128,128,0 128,128,1 256,128,2 256,256,3; do
    echo -n "$op tile $t: "; timeout -k 10 60 python scripts/op_bench.py $op --tile $t | grep gemm || echo "n/a"
  done
done
