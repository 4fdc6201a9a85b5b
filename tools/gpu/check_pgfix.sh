cd $GRAFT_REPO_ROOT
for m in side wire plain; do
  timeout -k 10 120 python -u tools/pg_capture_probe.py --rounds 30 --mode $m > gpurun_out/probe_$m.log 2>&1
  rc=$?
  echo "mode $m rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dp.py tests/test_gpu_rccl.py > gpurun_out/t_pgfix.log 2>&1
echo "dp tests rc=$?"
