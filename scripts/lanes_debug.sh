export TMPDIR=/tmp
T="tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread -k resnet_pipeline_matches_direct_model or lanes_match"
for i in 1 2 3; do echo -n "default $i: "; timeout -k 10 200 python -m pytest tests/test_gpu_pipeline.py -x -q -k "resnet_pipeline_matches_direct_model or lanes_match" 2>&1 | tail -1; done
for i in 1 2 3; do echo -n "admit0 $i: "; AIKO_GRAPH_ADMIT=0 timeout -k 10 200 python -m pytest tests/test_gpu_pipeline.py -x -q -k "resnet_pipeline_matches_direct_model or lanes_match" 2>&1 | tail -1; done
