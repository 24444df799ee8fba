#!/bin/bash
# round 5, call f: fbank (one-wave CMVN chains, fp32 log above the floor), the precise-text-backward
# parity variants, the shadow re-cast probe; c2 lines
source profiles/r5_lib.sh
O=gpurun_out/r5f; mkdir -p $O
step fbank 600 "${PYT[@]}" -s tests/test_kernels_gpu.py tests/test_torch_ops_gpu.py tests/test_data_gpu.py -k "fbank or feature" > $O/fbank.log 2>&1
step model 600 "${PYT[@]}" -s tests/test_model_gpu.py -k "golden_and_oracle" > $O/model.log 2>&1
step vprobe 300 python -u profiles/r5_version_probe.py > $O/vprobe.log 2>&1
for i in 1 2; do
  step bench_$i 300 python -u bench.py --no-cpu-baseline > $O/bench_$i.json 2> $O/bench_$i.err
done
