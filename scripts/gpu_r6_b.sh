#!/bin/bash
# Round 6: new / changed GPU tests first, then the full GPU suite, smoke, FA lab tests
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r6b}
mkdir -p $O
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $PT tests/test_fp16_gpu.py "tests/test_multirank_gpu.py::test_tp_oneshot_allreduce_matches_single_rank" "tests/test_multirank_gpu.py::test_zero1_other_optimizers_gather_params" > $O/new.log 2>&1 || { echo "FAIL new"; tail -40 $O/new.log; exit 1; }
tail -3 $O/new.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1 || { echo "FAIL suite"; tail -40 $O/suite.log; exit 1; }
tail -3 $O/suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "FAIL smoke"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
FLEETX_KERNELS_LIB=$(ls tools/fa_lab/_kernels*.so) timeout -k 10 300 $PT tools/fa_lab/test_fa_wave64_lab.py > $O/fa_lab.log 2>&1 || { echo "FAIL fa_lab"; tail -30 $O/fa_lab.log; exit 1; }
tail -2 $O/fa_lab.log
