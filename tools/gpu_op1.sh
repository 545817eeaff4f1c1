set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/op1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "into or chunk_edges or rmat12 or synthetic" > gpurun_out/op1/pytest.log 2>&1
rc=$?
tail -5 gpurun_out/op1/pytest.log
exit $rc
