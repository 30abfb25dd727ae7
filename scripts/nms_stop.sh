set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for s in ${STOPS:-1 2 3 4 99}; do
  AIKO_NMS_STOP=$s timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/nms$s -o run -- python3 scripts/nms_phases.py > gpurun_out/nms$s.log 2>&1
  echo "stop=$s"; python3 scripts/rocprof_summary.py gpurun_out/nms$s/run_results.db 2>&1 | grep -i "nms_${KER:-select}"
done
