# one GPU session: the -m gpu tests named in $GDD_TESTS (default: all), each step under its own limit
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu ${GDD_TESTS:-tests} > gpurun_out/t1.log 2>&1
rc=$?; tail -5 gpurun_out/t1.log; exit $rc
