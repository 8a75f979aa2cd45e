#!/bin/bash
# Round 6: multirank tests (deselected in r6g), then 6.7B step: this tree vs the round-start
# kernel library (interleaved, same box), fp16 O2 in the graph
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6h
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread "tests/test_multirank_gpu.py::test_layout_matches_single_rank_on_gpu" "tests/test_multirank_gpu.py::test_rccl_collective_forms_on_gpu" "tests/test_multirank_gpu.py::test_tp_oneshot_allreduce_matches_single_rank" "tests/test_multirank_gpu.py::test_zero1_other_optimizers_gather_params" > $O/mr.log 2>&1 || { echo FAIL; tail -30 $O/mr.log; exit 1; }
tail -1 $O/mr.log
run() {  # name, env..., -- args
  local name=$1; shift
  env "$@" timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
  echo $name $(grep -o '"value": [0-9.]*' $O/$name.log) $(grep -o '"ms_per_step": [0-9.]*' $O/$name.log) $(grep -o '"final_loss": [0-9.]*' $O/$name.log)
}
for r in 1 2; do
  run new_$r FLEETX_X=1
  run old_$r FLEETX_KERNELS_LIB=tools/bench_lab/_kernels_r6base.so
done
run fp16 FLEETX_BENCH_OVERRIDES=Engine.mix_precision.dtype=float16
grep -o '"hip_graph": [a-z]*' $O/fp16.log
