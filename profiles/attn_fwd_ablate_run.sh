set -e -o pipefail
P=scratch/abl
for m in 32 128 288 512; do
  STE_LIB=$P/libste_abl$m.so timeout -k 10 60 python3 -u profiles/attn_probe.py --no-bwd > gpurun_out/abl_$m.txt
done
STE_LIB=$P/libste_abl128.so timeout -k 10 60 python3 -u profiles/attn_probe.py --no-bwd --no-split > gpurun_out/abl_128ns.txt
