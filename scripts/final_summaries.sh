#!/bin/bash
# Copy a final session pair's evidence (gpurun_out/<A>, gpurun_out/<B>: scripts/sessions/
# r05_finalA.sh, r05_finalC.sh with TAG=<A>, TAG=<B>) into profiles/<A>, profiles/<B> and write the kstats, traffic and
# issue summaries bench.py quotes (each stamped with the digest the session recorded).
# usage: scripts/final_summaries.sh r05ia r05ib
set -e
A=$1; B=$2; cd "$(dirname "$0")/.."
G=gpurun_out/$A; P=profiles/$A; mkdir -p $P
cp $G/bench_c2_driver1.json $G/bench_c2_driver2.json $G/prof_c2.json $G/pytest.log $G/smoke.log $G/tree.txt $P/
cp $G/prof_c2/c2_kernel_stats.csv $G/prof_c2/c2_kernel_trace.csv $P/
cp $G/pmc_c2_fetch/f_counter_collection.csv $P/pmc_c2_fetch.csv
cp $G/pmc_c2_write/w_counter_collection.csv $P/pmc_c2_write.csv
cp $G/pmc_calib_fetch/f_counter_collection.csv $P/pmc_calib_fetch.csv
cp $G/pmc_calib_write/w_counter_collection.csv $P/pmc_calib_write.csv
cp $G/c2_sq1/p_counter_collection.csv $P/c2_sq1.csv
cp $G/c2_sq2/p_counter_collection.csv $P/c2_sq2.csv
H=gpurun_out/$B; Q=profiles/$B; mkdir -p $Q
cp $H/bench_c5.json $H/bench_c3.json $H/c5_new1.json $H/c5_new2.json $H/c5_nosplit1.json $H/c5_nosplit2.json $H/tree.txt $H/tutorial.log $Q/
for c in c5 c3; do
  cp $H/prof_$c/${c}_kernel_stats.csv $H/prof_$c/${c}_kernel_trace.csv $Q/
  cp $H/pmc_${c}_fetch/f_counter_collection.csv $Q/pmc_${c}_fetch.csv
  cp $H/pmc_${c}_write/w_counter_collection.csv $Q/pmc_${c}_write.csv
  cp $H/${c}_sq1/p_counter_collection.csv $Q/${c}_sq1.csv
  cp $H/${c}_sq2/p_counter_collection.csv $Q/${c}_sq2.csv
done
cp $H/prof_tut/tut_kernel_stats.csv $Q/
L2="VALU issue and dependency latency: the consumer's chain per iteration (scan, points, Girsanov trees, decision) and its wait for the producer's decision-dependent proposal; two waves per SIMD; W, F, H stay in registers/LDS across iterations (HBM traffic = the X/W proposal stores)"
L5="two balanced latency-bound waves per tile, one per SIMD (1 024 waves): producer (normals, u.W packets, W° whole lines) and consumer (H, F rows, recursion, X° whole lines); drawing every normal twice adds 560 µs per draw, the consumer's arithmetic twice 215 µs (profiles/r06h); loads, stores and hand-off alone 865 µs (r06g)"
L3="HBM throughput for its 6:3 read/write fp64 row mix with one wave per SIMD: a memory-only kernel of the same pattern runs 769-898 µs whatever the prefetch depth (profiles/r06f, scripts/c3_mem_probe.hip)"
K5='k_block_ps_pk<dmt::Lorenz<float>, float, 4'; K3='k_block<dmt::FHN<double>, double, 0'
python scripts/kstats_summary.py --trace $P/c2_kernel_trace.csv --kernel k_mcmc_resident_pc --config c2 --skip 5 --units-per-launch 20 --tree $P/tree.txt --command "rocprofv3 --kernel-trace --stats -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --repeats 0 --calls-iters 0 (dispatches: 5 one-iteration warm-up calls skipped; the timed call and the two event re-runs)" --out profiles/${A}_kstats_c2.json > /dev/null
python scripts/pmc_traffic.py --fetch $P/pmc_c2_fetch.csv --write $P/pmc_c2_write.csv --kernel k_mcmc_resident_pc --calib-fetch $P/pmc_calib_fetch.csv --calib-write $P/pmc_calib_write.csv --config c2 --units-per-launch 20 --skip 20 --tree $P/tree.txt --out profiles/${A}_traffic_c2.json > /dev/null
python scripts/issue_summary.py --kernel k_mcmc_resident_pc --config c2 --iters 20 --blocks 1024 --steps-per-block 500 --simds 1024 --skip 20 --csv $P/c2_sq1.csv $P/c2_sq2.csv --tree $P/tree.txt --command "rocprofv3 --pmc <SQ pass> -- python bench.py --steps 20 --warmup 20 --no-cpu-baseline --repeats 0 --calls-iters 0 (20 one-iteration warm-up dispatches skipped)" --bound valu-latency --limiter "$L2" --out profiles/${A}_issue_c2.json > /dev/null
python scripts/kstats_summary.py --trace $Q/c5_kernel_trace.csv --kernel "$K5" --config c5 --skip 3 --tree $Q/tree.txt --command "rocprofv3 --kernel-trace --stats -- python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline --calls-iters 0 --repeats 0 (the 3 warm-up draws skipped)" --out profiles/${B}_kstats_c5.json > /dev/null
python scripts/kstats_summary.py --trace $Q/c3_kernel_trace.csv --kernel "$K3" --config c3 --skip 3 --tree $Q/tree.txt --command "rocprofv3 --kernel-trace --stats -- python bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --calls-iters 0 --repeats 0 (the 3 warm-up draws skipped)" --out profiles/${B}_kstats_c3.json > /dev/null
python scripts/pmc_traffic.py --fetch $Q/pmc_c5_fetch.csv --write $Q/pmc_c5_write.csv --kernel "$K5" --calib-fetch $P/pmc_calib_fetch.csv --calib-write $P/pmc_calib_write.csv --calib-kernel 'k_stream<float>' --config c5 --skip 2 --tree $Q/tree.txt --out profiles/${B}_traffic_c5.json > /dev/null
python scripts/pmc_traffic.py --fetch $Q/pmc_c3_fetch.csv --write $Q/pmc_c3_write.csv --kernel "$K3" --calib-fetch $P/pmc_calib_fetch.csv --calib-write $P/pmc_calib_write.csv --calib-kernel 'k_stream<double>' --config c3 --skip 2 --tree $Q/tree.txt --out profiles/${B}_traffic_c3.json > /dev/null
python scripts/issue_summary.py --kernel "$K5" --config c5 --iters 1 --blocks 32768 --steps-per-block 2000 --simds 1024 --skip 2 --csv $Q/c5_sq1.csv $Q/c5_sq2.csv --tree $Q/tree.txt --command "rocprofv3 --pmc <SQ pass> -- python bench.py --config c5 --steps 4 --warmup 2 --no-cpu-baseline --calls-iters 0 --repeats 0 (the 2 warm-up draws skipped)" --bound hbm --limiter "$L5" --out profiles/${B}_issue_c5.json > /dev/null
python scripts/issue_summary.py --kernel "$K3" --config c3 --iters 1 --blocks 65536 --steps-per-block 1000 --simds 1024 --skip 2 --csv $Q/c3_sq1.csv $Q/c3_sq2.csv --tree $Q/tree.txt --command "rocprofv3 --pmc <SQ pass> -- python bench.py --config c3 --steps 4 --warmup 2 --no-cpu-baseline --calls-iters 0 --repeats 0 (the 2 warm-up draws skipped)" --bound hbm --limiter "$L3" --out profiles/${B}_issue_c3.json > /dev/null
python - "$A" "$B" <<'PY'
import csv, json, sys
A, B = sys.argv[1:3]
for n in (f'{A}_kstats_c2', f'{A}_traffic_c2', f'{A}_issue_c2', f'{B}_kstats_c5', f'{B}_kstats_c3',
          f'{B}_issue_c5', f'{B}_issue_c3', f'{B}_traffic_c5', f'{B}_traffic_c3'):
    d = json.load(open(f'profiles/{n}.json'))
    print(n, {k: (round(v, 3) if isinstance(v, float) else v) for k, v in d.items()
              if k in ('avg_us', 'median_us', 'traffic_bytes_per_unit', 'simd_valu_busy',
                       'valu_active_frac', 'wait_any_frac', 'csrc_sha16')})
rows = list(csv.DictReader(open(f'profiles/{B}/tut_kernel_stats.csv')))
print('tutorial kernel ms per iteration', round(sum(float(r['TotalDurationNs']) for r in rows) / 1e6 / 300, 3))
PY
