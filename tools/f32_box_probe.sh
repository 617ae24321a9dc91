#!/bin/bash
# Round 6: the float32 paths' time per box.  On one box:
# its GPU identity, bare 16-B store bandwidth (tools/write_bw), st_step_f32
# and the f32 rollout graph-replayed (tools/ab_f32.py), and the f32 rollout
# at 100 and 400 steps per launch with events per launch (tools/ab_rollout.py).
# Run it in two separate gpurun calls to compare boxes.
#   gpurun -- bash tools/f32_box_probe.sh TAG   -> gpurun_out/f32box_TAG.txt
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; export TMPDIR=/tmp; mkdir -p gpurun_out
O="gpurun_out/f32box_${1:-a}.txt"
{
  timeout -k 10 60 python -c "import torch; p = torch.cuda.get_device_properties(0); print('box', p.uuid, 'pci_bus', getattr(p, 'pci_bus_id', None))" &&
  timeout -k 10 120 ./tools/write_bw &&
  timeout -k 10 120 python tools/ab_f32.py &&
  timeout -k 10 120 python tools/ab_rollout.py 100 10 f32 &&
  timeout -k 10 120 python tools/ab_rollout.py 400 3 f32 &&
  timeout -k 10 120 python tools/ab_f32.py
} > "$O" 2>&1
rc=$?
grep -v amdgpu.ids "$O"
exit $rc
