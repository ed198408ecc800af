cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=15 --timeout 400 --timeout-method thread > gpurun_out/r03_gputests.log 2>&1; rc=$?
echo "tests rc=$rc" >> gpurun_out/r03_gputests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/r03_bench.log 2>&1
