#!/bin/bash
# round 6, session A: GPU suite on the new tree (TD aux base hoisted, persistent TD opt-in,
# consumer histories through LDS), then the C2 headline A/B over the consumer build switches:
# def (NST_OPAQUE=1, HIST_LDS=1), base (0, 0), nst (1, 0), hist (0, 1); rocprofv3 for def, base
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06a; mkdir -p $O
python scripts/provenance.py > $O/tree.txt
S=("timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1")
for r in 1 2; do
  for v in def base nst hist; do
    if [ $v = def ]; then LP=$PWD/diffusionmcmctools.jl_amd/libdmt.so; else LP=$PWD/build_variants/libdmt_$v.so; fi
    S+=("DMT_LIB_PATH=$LP timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --calls-iters 0 --repeats 20 > $O/c2_${v}_$r.json 2> $O/c2_${v}_$r.err")
  done
done
for v in def base; do
  if [ $v = def ]; then LP=$PWD/diffusionmcmctools.jl_amd/libdmt.so; else LP=$PWD/build_variants/libdmt_$v.so; fi
  S+=("DMT_LIB_PATH=$LP timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o c2 --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --calls-iters 0 --repeats 20 > $O/prof_$v.json 2> $O/prof_$v.log")
done
# the tutorial workload (one FHN block, two 10^4-step recursions per iteration): kernel trace
# and SQ passes of k_block_wave (attribute its ≈78 ns per serial step)
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU_FMA_F64"
P3="SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_SALU SQ_INSTS_BRANCH SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64"
S+=("timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tut_kt -o tut --output-format csv -- python examples/fhn_gamma_inference.py --steps 60 --burn-in 10 > $O/tut_kt.log 2>&1")
for P in 1 2 3; do
  eval "PC=\$P$P"
  S+=("timeout -s KILL 120 rocprofv3 --pmc $PC -d $O/tut_p$P -o p --output-format csv -- python examples/fhn_gamma_inference.py --steps 20 --burn-in 5 > $O/tut_p$P.log 2>&1")
done
scripts/gpu_session.sh "${S[@]}"
tail -2 $O/pytest.log
for f in $O/c2_*.json; do python -c "import json;d=json.load(open('$f'));print('$f', round(d['value']/1e10,4), round(d['repeats']['value_median']/1e10,4), round(d['roofline']['kernel_avg_us'],2))"; done
for v in def base; do python -c "
import csv,glob,statistics
f=glob.glob('$O/prof_$v/*kernel_trace.csv')[0]
d=[(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3 for r in csv.DictReader(open(f)) if 'k_mcmc_resident_pc' in r['Kernel_Name']]
d=d[5:]
print('$v', len(d), round(statistics.median(d),2), round(min(d),2))"; done
python scripts/sq_summary.py k_block_wave 10000 $(find $O/tut_p1 $O/tut_p2 $O/tut_p3 -name "*counter_collection.csv") > $O/tut_sq.txt 2>&1
head -20 $O/tut_sq.txt
