#!/bin/bash
# round 5, third GPU call: the precise text backward (fp32 text attention backward, split-bf16 dY
# operands, fp32 dO and bias sums, split dW operands) and the side-stream text collectives:
# kernel + model parity tests, determinism, public-API, DP tests, then c2 lines
source profiles/r5_lib.sh
O=gpurun_out/r5c; mkdir -p $O
step kern 600 "${PYT[@]}" -s tests/test_kernels_gpu.py -k "attention_f32 or adamw" > $O/kern.log 2>&1
step model 900 python -u -m pytest -v -s --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_model_gpu.py tests/test_torch_ops_gpu.py tests/test_determinism_gpu.py tests/test_dist_gpu.py tests/test_rccl_gpu.py tests/test_checkpoint_gpu.py tests/test_eval_gpu.py > $O/model.log 2>&1
for i in 1 2; do
  step bench_$i 300 python -u bench.py --no-cpu-baseline > $O/bench_$i.json 2> $O/bench_$i.err
done
