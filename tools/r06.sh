# round-6 GPU session driver: bash tools/r06.sh <tag> [suite] [bench] [tp]
set -o pipefail
mkdir -p gpurun_out
T=$1; shift
O=gpurun_out/$T
for step in "$@"; do
  case $step in
    suite)
      timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O.pytest.log 2>&1 || { echo pytest failed; grep -E "FAILED|Error" $O.pytest.log | head -20; exit 1; }
      tail -1 $O.pytest.log
      timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O.smoke.log 2>&1 || { echo smoke failed; tail $O.smoke.log; exit 1; }
      tail -1 $O.smoke.log ;;
    bench)
      timeout -k 10 300 python -u bench.py $BENCH_ARGS > $O.bench.json 2> $O.bench.err || { echo bench failed; tail $O.bench.err; exit 1; }
      python -c "import json; d=json.load(open('$O.bench.json')); print('bench', round(d['value']), round(d['ms_per_step'],1), round(d['mfu'],4), round(d['roofline']['frac'],4))" ;;
    tp)
      for c in ${TPCHUNKS:-0 2}; do
        PICOTRON_TP_SP_CHUNKS=$c timeout -k 10 200 python -u bench.py --tp-proxy 8 --steps 5 > $O.tp$c.json 2> $O.tp$c.err || { echo tp$c failed; tail -5 $O.tp$c.err; exit 1; }
        python -c "import json; d=json.load(open('$O.tp$c.json')); print('tp8 chunks $c', round(d['value']), round(d['ms_per_microbatch'],2), round(d['eager_ms_per_microbatch'],2), d['launch'], d.get('graph_note'), d['config']['sp_chunks'])"
      done ;;
  esac
done
