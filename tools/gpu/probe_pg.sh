# ProcessGroupNCCL watchdog vs capture: one process per mode, each under its own limit; the first
# abort ends the script (the modes run from the DataParallel-like forms to the bf16 wire)
cd $GRAFT_REPO_ROOT
for m in plain async side wire; do
  timeout -k 10 120 python -u tools/pg_capture_probe.py --rounds 30 --mode $m > gpurun_out/probe_$m.log 2>&1
  rc=$?
  echo "mode $m rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
