cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_cpp_host_blocks.py -k teacher > gpurun_out/t_it6.log 2>&1
rc=$?
grep -E "^\(|segments|fault|PASSED|FAILED|Error" gpurun_out/t_it6.log | head -90
exit $rc
