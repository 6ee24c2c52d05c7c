cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > gpurun_out/r06b_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r06b_pytest.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06b_smoke.log 2>&1; tail -1 gpurun_out/r06b_smoke.log
