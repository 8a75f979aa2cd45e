#!/bin/bash
# Round 6 end: full GPU suite + smoke + default bench on the final tree
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r6final}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
grep '"metric"' $O/bench.log | cut -c1-220
FLEETX_KERNELS_LIB=$(ls tools/fa_lab/_kernels.cpython*.so) timeout -k 10 300 python -u -m pytest tools/fa_lab/test_fa_wave64_lab.py -x -q --timeout 120 --timeout-method thread > $O/fa_lab.log 2>&1 || { tail -20 $O/fa_lab.log; exit 1; }
tail -1 $O/fa_lab.log
