set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$1/gputest.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/$1/bench.json 2> gpurun_out/$1/bench.err || exit $?
