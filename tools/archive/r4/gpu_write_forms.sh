# Round-4 A/B of the write pass's forms after the pass-based sync: 4 lanes per subsequence
# (k_write4) or one (k_write, VF_JPEG_WRITE4=0), chunked rows (VF_JPEG_CHUNKS=1) or a cleared
# buffer (0), on hard 1080p and 4K scenes; resident batches, two reps each.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in "1 auto" "0 1" "0 0"; do
    set -- $cfg
    for c in "hard 1080p" "scene 4k"; do
      set -- $cfg $c
      envs="VF_JPEG_WRITE4=$1"; [ "$2" != auto ] && envs="$envs VF_JPEG_CHUNKS=$2"
      env $envs timeout -k 10 200 python3 tools/jpeg_bench.py --sizes $4 --batch 32 --iters 10 --cpu-seconds 0 --resident-only --content $3 --out gpurun_out/wf.jsonl > gpurun_out/wf.log 2>&1 || { echo WF_FAILED; tail -20 gpurun_out/wf.log; exit 1; }
      python3 -c "import json; d=json.loads(open('gpurun_out/wf.jsonl').read().splitlines()[-1]); print('rep $rep', '$envs', '$3 $4', d['gpu_resident_fps'], d['parity_vs_oracle'], d['stages_ms']['huffman_write'])"
    done
  done
done
