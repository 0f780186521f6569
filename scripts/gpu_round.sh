cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
bash scripts/profile_stream.sh > gpurun_out/prof.log 2>&1
echo exit $?
