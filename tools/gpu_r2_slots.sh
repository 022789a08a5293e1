# Engine slot size A/B for the host->host paths (VF_SLOT_BYTES), 2 interleaved rounds.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/r2_e2e_slots.jsonl
for r in 1 2; do
  for sb in 16777216 33554432 67108864; do
    VF_SLOT_BYTES=$sb timeout -k 10 120 python -u tools/e2e_probe.py | sed "s/^{/{\"slot_bytes\": $sb, /" >> gpurun_out/r2_e2e_slots.jsonl || { echo E2E_FAILED; exit 1; }
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r2_e2e_slots.jsonl"):
    d = json.loads(l)
    print(d["slot_bytes"] >> 20, "MiB", d["size"], "pageable", d["pageable_GBps_each_way"], "pinned", d["pinned_GBps_each_way"], "pipelined", d["pinned_pipelined_GBps_each_way"])
PY
