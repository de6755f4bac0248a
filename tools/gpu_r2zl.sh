#!/bin/bash
# Round-2 GPU pass zl: HIP runtime launch knobs vs the dependent-launch gap (launch_gap.py) and the bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r2zl
bash tools/gpu_steps.sh \
  "120|r2zl/gap_default|python -u tools/launch_gap.py && python -u bench.py --steps 300 --warmup 30" \
  "120|r2zl/gap_devkernarg1|HIP_FORCE_DEV_KERNARG=1 python -u tools/launch_gap.py && HIP_FORCE_DEV_KERNARG=1 python -u bench.py --steps 300 --warmup 30" \
  "120|r2zl/gap_devkernarg0|HIP_FORCE_DEV_KERNARG=0 python -u tools/launch_gap.py && HIP_FORCE_DEV_KERNARG=0 python -u bench.py --steps 300 --warmup 30" \
  "120|r2zl/gap_pktcap1|DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 python -u tools/launch_gap.py && DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 python -u bench.py --steps 300 --warmup 30" \
  "120|r2zl/gap_pktcap0|DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 python -u tools/launch_gap.py && DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 python -u bench.py --steps 300 --warmup 30" \
  "120|r2zl/gap_default2|python -u tools/launch_gap.py && python -u bench.py --steps 300 --warmup 30"
