#!/bin/bash
# One parameterised driver for the GPU-box sessions (replaces the round-2 one-off lease scripts).
# Run from the repo root ON THE BOX (through gpurun):   bash tools/gpu.sh <tag> <step>[,<step>...] [k=v ...]
#
# steps (run in the order given; the first failure ends the call -- no retries on the GPU):
#   suite        pytest -m gpu (whole suite; TESTS=... files / node ids, TESTK=... a -k expression), then smoke()
#   bench        bench.py N=1 (BENCH_RUNS=2 lines), default arguments
#   prof         rocprofv3 --kernel-trace --stats of bench.py --steps 2 (kernel table -> profiles via tools/prof_summary.py)
#   pmc          GEMM/all-kernel HBM traffic: separate FETCH_SIZE and WRITE_SIZE passes over bench.py --grad-acc 2
#   pmcx         extra counter sets over bench.py --grad-acc 1 (SQ busy/VALU/MFMA, TCC hit/miss/EA reads)
#   configs      llama + tp + cp: Llama-2-7B 1-GPU bench, TP=8 proxy, CP=8 proxy (each also a step)
#   gloo2        bench.py --gpus 2 --backend gloo rehearsal (2 ranks on cuda:0)
#   pp2          bench.py --gpus 2 --pp 2 --backend gloo rehearsal of the pipeline engine (config 4's 1F1B)
#   grid8        bench.py --gpus 8 --backend gloo: DP=8, TP=8, config 4 (llama2-7b tp2 pp2), config 5 (cp8 32k)
#   dp           bench.py --dp-bucket fp32 / bf16 vs plain (the per-GPU DP cost)
#   dpprof       rocprofv3 kernel table of bench.py --dp-bucket (GT=fp32|bf16)
#   gemm         tools/gemm_bench.py --brief (GTILES=12,13,14, GEMM_ARGS)
#   attn         tools/attn_bench.py d64 and d128 (OLD=<lib> for an in-process A/B; ATTN64_ARGS for the d64 run)
#   pmcattn      attention PMC passes (ATTN_ARGS="--B 1 --S 4096 --H 32 --D 128" for d128)
#   norm         tools/norm_bench.py (OLD=<lib> for an A/B)
#   tpprof       rocprofv3 kernel trace of the TP=8 proxy (PROXY="--tp-proxy 8" or "--cp-proxy 8 --model ...")
#   counters     rocprofv3 -L: the counters this box's gfx950 exposes (e.g. for HBM vs Infinity-Cache reads)
#   mall         TCC_EA0_RDREQ vs TCC_EA0_RDREQ_DRAM on a cold and a warm (Infinity-Cache) read (tools/mall_probe.py)
#   envab        whole-step A/B of two (or three: C=...) env settings: A="X=0" B="X=1" ROUNDS=3
#   libab        whole-step A/B of library builds swapped in place: LIBS=a.so,b.so ROUNDS=2
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=$1; STEPS=$2; shift 2
for kv in "$@"; do export "$kv"; done
LIB=picotron_amd/lib/libpicotron_hip.so
O=gpurun_out/$T

jline() {  # print a bench JSON line's headline fields
  python -c "import json,sys; d=json.load(open('$1')); r=d.get('roofline') or {}; print('$2', round(d['value']), round(d.get('ms_per_step', d.get('ms_per_microbatch', 0)),1), round(d.get('mfu', d.get('mfu_upper_bound', 0)) or 0,4), round(r.get('frac', 0) or 0,3))"
}

step_suite() {
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} ${TESTK:+-k "$TESTK"} -m gpu -x -q --timeout 300 --timeout-method thread > $O.pytest.log 2>&1 || { echo pytest failed; grep -E "Error|FAILED|assert" $O.pytest.log | head -30; return 1; }
  tail -1 $O.pytest.log
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O.smoke.log 2>&1 || { echo smoke failed; tail $O.smoke.log; return 1; }
  tail -1 $O.smoke.log
}

step_bench() {
  for i in $(seq 1 ${BENCH_RUNS:-1}); do
    timeout -k 10 300 python -u bench.py $BENCH_ARGS > $O.bench$i.json 2> $O.bench$i.err || { echo bench failed; tail $O.bench$i.err; return 1; }
    jline $O.bench$i.json bench
  done
}

step_prof() {
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O.prof -o k -- python -u bench.py --steps 2 --warmup 1 --cpu-tokens 0 > $O.prof.log 2>&1 || { echo prof failed; tail $O.prof.log; return 1; }
  gzip -f $O.prof/k_kernel_trace.csv
  python tools/prof_summary.py --trace $O.prof/k_kernel_trace.csv.gz --steps 3 > $O.kernels.md || true
}

step_pmc() {
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O.pmc1 -o f -- python -u bench.py --steps 1 --warmup 0 --grad-acc 4 --cpu-tokens 0 --no-probe > $O.pmc1.log 2>&1 || { echo pmc1 failed; return 1; }
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O.pmc2 -o w -- python -u bench.py --steps 1 --warmup 0 --grad-acc 4 --cpu-tokens 0 --no-probe > $O.pmc2.log 2>&1 || { echo pmc2 failed; return 1; }
  python tools/traffic_summary.py $O.pmc1/f_counter_collection.csv $O.pmc2/w_counter_collection.csv $O.gemm_traffic.json \
    '{"model": "SmolLM-1.7B", "layers": 15, "micro_batch": 4, "seq_len": 1024, "parallelism": "dp1"}' $LIB
}

step_pmcx() {
  local i=0
  for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" ${PMCX_EXTRA}; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d $O.pmcx$i -o c -- python -u bench.py --steps 1 --warmup 0 --grad-acc 1 --cpu-tokens 0 --no-probe > $O.pmcx$i.log 2>&1 || { echo "pmcx $i failed"; tail -3 $O.pmcx$i.log; return 1; }
  done
}

step_llama() {
  timeout -k 10 400 python -u bench.py --model llama2-7b --grad-acc 8 --steps 2 --warmup 1 --cpu-tokens 0 > $O.llama.json 2> $O.llama.err || { echo llama failed; tail $O.llama.err; return 1; }
  jline $O.llama.json llama2-7b
}

step_tp() {
  timeout -k 10 200 python -u bench.py --tp-proxy 8 --steps 3 > $O.tpproxy.json 2> $O.tpproxy.err || { echo tpproxy failed; tail $O.tpproxy.err; return 1; }
  jline $O.tpproxy.json tp8-proxy
}

step_cp() {
  timeout -k 10 300 python -u bench.py --cp-proxy 8 --model llama2-7b --seq 32768 --mbs 1 --steps 3 $CP_ARGS > $O.cpproxy.json 2> $O.cpproxy.err || { echo cpproxy failed; tail $O.cpproxy.err; return 1; }
  python -c "import json; d=json.load(open('$O.cpproxy.json')); print('cp8 proxy', round(d['value']), round(d['modelled_with_mesh_comm_tokens_per_s_per_gpu']), {k: round(v,2) for k,v in d['critical_rank_layer_ms_with_comm'].items()}, d['bound'], d['comm']['mesh']['exposed_ms'], round(d['roofline']['fwd_frac'],3), round(d['roofline']['bwd_frac'],3))"
}

step_configs() { step_llama && step_tp && step_cp; }

step_gloo2() {
  timeout -k 10 400 python -u bench.py --gpus 2 --backend gloo --steps 1 --warmup 1 --grad-acc 4 > $O.gloo2.json 2> $O.gloo2.err || { echo gloo2 failed; tail -20 $O.gloo2.err; return 1; }
  [ $(wc -l < $O.gloo2.json) = 1 ] || { echo "gloo2: stdout is not one line"; return 1; }
  python -c "import json; d=json.load(open('$O.gloo2.json')); print('gloo2', d['n_gpus'], d['ranks'], d['backend'], d['config']['parallelism'], round(d['value']))"
}

step_pp2() {
  timeout -k 10 400 python -u bench.py --gpus 2 --pp 2 --backend gloo --steps 1 --warmup 1 --grad-acc 4 --cpu-tokens 0 ${PP_ARGS} > $O.pp2.json 2> $O.pp2.err || { echo pp2 failed; tail -20 $O.pp2.err; return 1; }
  [ $(wc -l < $O.pp2.json) = 1 ] || { echo "pp2: stdout is not one line"; return 1; }
  python -c "import json; d=json.load(open('$O.pp2.json')); print('pp2', d['n_gpus'], d['ranks'], d['backend'], d['config']['parallelism'], round(d['value']), d['final_loss'])"
}

step_grid8() {   # every 8-rank grid the driver's 8-GPU run can launch, assembled once over gloo on cuda:0
  local n=0
  while IFS='|' read -r tag args; do
    [ -n "$tag" ] || continue
    n=$((n+1))
    timeout -k 10 ${GRID8_TIMEOUT:-420} python -u bench.py --gpus 8 --backend gloo --steps 1 --warmup 1 --cpu-tokens 0 $args > $O.grid8_$tag.json 2> $O.grid8_$tag.err || { echo "grid8 $tag failed"; tail -20 $O.grid8_$tag.err; return 1; }
    [ $(wc -l < $O.grid8_$tag.json) = 1 ] || { echo "grid8 $tag: stdout is not one line"; return 1; }
    python -c "import json; d=json.load(open('$O.grid8_$tag.json')); print('grid8 $tag', d['n_gpus'], d['ranks'], d['backend'], d['config']['parallelism'], round(d['value']), d['final_loss'])"
  done <<< "${GRID8:-dp8|--layers 2 --grad-acc 2
tp8|--tp 8 --layers 2 --grad-acc 2
cfg4|--model llama2-7b --tp 2 --pp 2 --layers 4 --grad-acc 4
cfg5|--model llama2-7b --cp 8 --seq 32768 --mbs 1 --layers 2 --grad-acc 1}"
}

step_dp() {
  for gt in fp32 bf16; do
    timeout -k 10 300 python -u bench.py --dp-bucket --grad-type $gt --steps 3 --cpu-tokens 0 > $O.dp_$gt.json 2>/dev/null || { echo dp $gt failed; return 1; }
    jline $O.dp_$gt.json dp-bucket-$gt
  done
  timeout -k 10 300 python -u bench.py --steps 3 --cpu-tokens 0 > $O.plain.json 2>/dev/null || { echo plain failed; return 1; }
  jline $O.plain.json plain
}

step_dpprof() {   # kernel table of the DP path on a 1-rank RCCL group (fp32 main_grad sinks), beside prof's plain table
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O.dpprof -o k -- python -u bench.py --dp-bucket --grad-type ${GT:-fp32} --steps 2 --warmup 1 --cpu-tokens 0 > $O.dpprof.log 2>&1 || { echo dpprof failed; tail $O.dpprof.log; return 1; }
  gzip -f $O.dpprof/k_kernel_trace.csv
  python tools/prof_summary.py --trace $O.dpprof/k_kernel_trace.csv.gz --steps 3 > $O.dpkernels.md || true
}

step_gemm() {    # tools/gemm_bench.py over the layer's shapes (GTILES, GEMM_ARGS e.g. "--tp 8")
  timeout -k 10 300 python -u tools/gemm_bench.py --tiles ${GTILES:-12,13,14} --brief $GEMM_ARGS > $O.gemm.log 2>&1 || { echo gemm failed; tail $O.gemm.log; return 1; }
  cat $O.gemm.log
}

step_attn() {
  local old=${OLD:+--old $OLD}
  timeout -k 10 200 python -u tools/attn_bench.py --rounds ${ROUNDS:-4} $old ${ATTN64_ARGS} > $O.attn_d64.log 2>&1 || { echo attn d64 failed; tail -30 $O.attn_d64.log; return 1; }
  cat $O.attn_d64.log
  timeout -k 10 200 python -u tools/attn_bench.py --rounds ${ROUNDS:-4} --B 1 --S 4096 --D 128 $old > $O.attn_d128.log 2>&1 || { echo attn d128 failed; tail -30 $O.attn_d128.log; return 1; }
  cat $O.attn_d128.log
}

step_pmcattn() {
  local i=0
  for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv --kernel-include-regex attn -d $O.pmca$i -o a -- python -u tools/attn_bench.py --reps 5 $ATTN_ARGS > $O.pmca$i.log 2>&1 || { echo "pmcattn $i failed"; tail -3 $O.pmca$i.log; return 1; }
  done
}

step_norm() {
  timeout -k 10 120 python -u tools/norm_bench.py ${OLD:+--old $OLD} > $O.norm.log 2>&1 || { echo norm failed; tail $O.norm.log; return 1; }
  grep -v "^$" $O.norm.log | tail -8
}

step_tpprof() {
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O.tpprof -o k -- python -u bench.py ${PROXY:---tp-proxy 8} --steps 3 > $O.tpprof.log 2>&1 || { echo tpprof failed; tail $O.tpprof.log; return 1; }
  gzip -f $O.tpprof/k_kernel_trace.csv
  tail -1 $O.tpprof.log
}

step_counters() {
  timeout -k 10 120 rocprofv3 -L > $O.counters.txt 2>&1 || { echo counters failed; tail $O.counters.txt; return 1; }
  grep -ciE "TCC_EA|MALL|DRAM|HBM" $O.counters.txt || true
}

step_mall() {
  timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum --kernel-include-regex reduce --output-format csv -d $O.mall -o m -- python -u tools/mall_probe.py > $O.mall.log 2>&1 || { echo mall failed; tail -3 $O.mall.log; return 1; }
  python - "$O.mall/m_counter_collection.csv" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
per = collections.defaultdict(dict)
for r in rows:
    per[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
for d in sorted(per):
    print(d, {k: int(v) for k, v in sorted(per[d].items())})
PY
}

step_envab() {
  for i in $(seq 1 ${ROUNDS:-3}); do
    for v in A B ${C:+C}; do
      if [ $v = A ]; then E=$A; elif [ $v = B ]; then E=$B; else E=$C; fi
      env $E timeout -k 10 300 python -u bench.py --cpu-tokens 0 --steps 3 $BENCH_ARGS > $O.$v$i.json 2>/dev/null || { echo "bench $E failed"; return 1; }
      jline $O.$v$i.json "$E"
    done
  done
}

step_libab() {
  IFS=, read -ra L <<< "$LIBS"
  for f in "${L[@]}"; do [ -f "$f" ] || { echo "missing $f on the box"; return 1; }; done
  [ $(md5sum "${L[@]}" | cut -d' ' -f1 | sort -u | wc -l) -eq ${#L[@]} ] || { echo "identical builds in $LIBS"; return 1; }
  cp $LIB $O.orig.so
  for i in $(seq 1 ${ROUNDS:-2}); do
    for f in "${L[@]}"; do
      cp "$f" $LIB || return 1
      n=$(basename $f .so)
      timeout -k 10 300 python -u bench.py --cpu-tokens 0 --steps 3 $BENCH_ARGS > $O.${n}_$i.json 2>/dev/null || { echo "bench $n failed"; cp $O.orig.so $LIB; return 1; }
      jline $O.${n}_$i.json $n
    done
  done
  cp $O.orig.so $LIB && rm -f $O.orig.so
}

IFS=, read -ra S <<< "$STEPS"
for s in "${S[@]}"; do
  echo "== $s"
  step_$s || exit 1
done
find gpurun_out -name "*.db" -delete
echo done
