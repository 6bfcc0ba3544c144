#!/bin/bash
# Round 4: the bench line's timing events with default flags vs hipEventDisableSystemFence
# (0x20000000) vs hipEventReleaseToDevice (0x40000000): host time per C2 call
# (scripts/host_timing.py) and the driver-command bench line, interleaved.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04p}
mkdir -p $O
BC="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --repeats 10 --calls-iters 0"
for r in 1 2; do
  for f in 0 0x20000000 0x40000000; do
    DMT_EVENT_FLAGS=$f timeout -k 10 120 python scripts/host_timing.py > $O/host_${f}_$r.json 2> $O/host_${f}_$r.err || exit $?
    DMT_EVENT_FLAGS=$f timeout -k 10 150 $BC > $O/bench_${f}_$r.json 2> $O/bench_${f}_$r.err || exit $?
  done
done
echo done
