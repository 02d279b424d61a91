# round-4 diagnostics (one GPU call): the GPU suite's first failure in isolation and in order,
# then the autograd step's cost breakdown.  Every step under its own time limit; an abnormal
# exit (fault, abort, timeout) ends the script.
set -u
mkdir -p gpurun_out
ok() { case $1 in 0|1) return 0;; *) return 1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_mrg32k3a.py -m gpu -x -v --tb=long -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/diag_mrg.log 2>&1
rc=$?; echo "mrg rc=$rc"; ok $rc || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --tb=long -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/diag_full.log 2>&1
rc=$?; echo "full rc=$rc"; ok $rc || exit $rc
timeout -k 10 300 python -u tools/autograd_cost.py > gpurun_out/autograd_cost.json 2> gpurun_out/autograd_cost.err
rc=$?; echo "autograd_cost rc=$rc"; exit $rc
