#!/bin/bash
# round 6, call a: the new bench-plan parity tests first (GEMM epilogue specs at >= 240 tiles, the
# b = 64 vs 16 x 4 plan equivalence, the full-size draws and 8-phase-plan instances), then the whole
# GPU suite with its parity prints (profiles/r6_parity.txt), smoke, one c2 bench line
source profiles/r6_lib.sh
O=gpurun_out/r6a; mkdir -p $O
step new_tests 900 python -u -m pytest tests/test_gemm_specs_gpu.py tests/test_plan_equivalence_gpu.py tests/test_fullsize_gpu.py -m gpu -v -s -p no:cacheprovider --timeout 600 --timeout-method thread > $O/new_tests.log 2>&1
step gpu_tests 1100 python -u -m pytest tests -m gpu -v -s -p no:cacheprovider --timeout 900 --timeout-method thread --deselect tests/test_fullsize_gpu.py --deselect tests/test_gemm_specs_gpu.py --deselect tests/test_plan_equivalence_gpu.py > $O/gpu_tests.log 2>&1
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
step bench_c2 600 python -u bench.py --steps 20 --warmup 5 > $O/bench_c2.json 2> $O/bench_c2.err
# epilogue store-burst experiment: workgroup groups started 1/G of a tile apart (-DSTE_GEMM_SKEW=G builds)
for L in libste_ab libste_skew2 libste_skew4; do
  STE_LIB=$PWD/speech_transcript_embeddings_amd/$L.so step probe_$L 300 python -u profiles/gemm_probe.py --iters 30 > $O/probe_$L.jsonl 2>&1
done
# the packed-fp32 LayerNorm defect re-checked on this toolchain: shipped libste.so
# (packed fp32 off) vs libste_pk.so (layernorm.hip with packed fp32, everything else identical)
for L in libste libste_pk; do
  STE_LIB=$PWD/speech_transcript_embeddings_amd/$L.so MODES=idle,gemm REPS=40 step det_ln_$L 300 python -u profiles/det_ln.py > $O/det_ln_$L.log 2>&1
done
