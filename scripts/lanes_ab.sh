export TMPDIR=/tmp
T="tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread -k lanes_match"
echo "default:"; timeout -k 10 300 python -m pytest $T 2>&1 | tail -1
echo "attn10:"; AIKO_ATTN_VARIANT=10 timeout -k 10 300 python -m pytest $T 2>&1 | tail -1
echo "admit0:"; AIKO_GRAPH_ADMIT=0 timeout -k 10 300 python -m pytest $T 2>&1 | tail -1
echo "both:"; AIKO_GRAPH_ADMIT=0 AIKO_ATTN_VARIANT=10 timeout -k 10 300 python -m pytest $T 2>&1 | tail -1
