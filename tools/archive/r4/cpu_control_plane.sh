# Control-plane headroom: tools/distributor_overhead.py --no-copy with N = 1, 2,
# 4, 8 in-place echo workers (no GPU, no host copies) at configs[2] (4K, batch 16, shard),
# configs[3] (480p/1080p/4K interleaved, batch 16, pull) and the JPEG 1080p leg (182 KB, batch 32,
# pull).  Runs on the GPU box for its CPU share; touches no GPU.
set -o pipefail
mkdir -p gpurun_out
OUT=${1:-gpurun_out/control_plane.jsonl}
rm -f $OUT
for n in 1 2 4 8; do
  timeout -k 10 120 python -u tools/distributor_overhead.py --no-copy --workers $n --policy shard --bytes 24883200 --batch 16 --frames $((4000 * n)) --group 8 --out $OUT | tail -1 || exit 1
  timeout -k 10 120 python -u tools/distributor_overhead.py --no-copy --workers $n --policy pull --mixed --batch 16 --frames $((4000 * n)) --group 8 --out $OUT | tail -1 || exit 1
  timeout -k 10 120 python -u tools/distributor_overhead.py --no-copy --workers $n --policy pull --bytes 181876 --batch 32 --frames $((8000 * n)) --group 16 --out $OUT | tail -1 || exit 1
done
echo CP_OK
