#!/bin/bash
# Variants of tools/stall_probe.py (outputs under gpurun_out/stall): the loop
# on 1 or 2 streams, the null stream or not, more hardware queues, no loop,
# an idle gap; XRT_SIZING_PROFILE=2 times the sizing path's calls on the host
# without synchronising (=1 synchronises each step and hides the stall).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/stall
mkdir -p $o
export XRT_SIZING_PROFILE=${XRT_SIZING_PROFILE:-2}
run() { name=$1; shift; timeout -k 10 120 python tools/stall_probe.py "$@" > $o/$name.json 2> $o/$name.err || exit 1; }
run a_2null --streams 2 --null
run b_2own --streams 2
run c_1null --streams 1 --null
run d_1own --streams 1
GPU_MAX_HW_QUEUES=16 run e_2null_q16 --streams 2 --null
run f_noloop --streams 2 --null --frames 0
run g_idle --streams 2 --null --idle-ms 50
run h_2null_again --streams 2 --null
# the pinned-ring D2H's copy threads (0: pageable hipMemcpy)
XRT_D2H_THREADS=0 run k_thr0 --frames 0
XRT_D2H_THREADS=4 run j_thr4 --frames 0
XRT_D2H_THREADS=16 run i_thr16 --frames 0
