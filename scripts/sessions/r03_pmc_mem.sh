#!/bin/bash
# Memory-path counters of the C5 and C3 draw kernels: UTCL1 translation, TCP->TCC request
# latency, TCC->EA (HBM) request queue levels, TA/TD busy.  One pass per counter group.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03pmc}
mkdir -p $O
P1="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_PENDING_STALL_CYCLES_sum"
P2="TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"
P3="TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_WRREQ_sum"
P4="TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE GRBM_COUNT"
steps=()
for cfg in c5 c3; do
  B="python bench.py --config $cfg --steps 2 --warmup 1 --repeats 0 --no-cpu-baseline"
  i=1
  for P in "$P1" "$P2" "$P3" "$P4"; do
    steps+=("timeout -s KILL 170 rocprofv3 --pmc $P -d $O/${cfg}_p$i -o p --output-format csv -- $B > $O/${cfg}_p$i.log 2>&1")
    i=$((i+1))
  done
done
scripts/gpu_session.sh "${steps[@]}"
