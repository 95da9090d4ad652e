set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r06a
true; rc=0
tail -25 $O.pytest.log
[ $rc = 0 ] || exit $rc
for c in 1 2 4; do
  PICOTRON_TP_SP_CHUNKS=$c timeout -k 10 200 python -u bench.py --tp-proxy 8 --steps 5 > $O.tp$c.json 2> $O.tp$c.err || { echo tp$c failed; tail $O.tp$c.err; exit 1; }
  python -c "import json; d=json.load(open('$O.tp$c.json')); print('tp8 chunks $c', round(d['value']), round(d['ms_per_microbatch'],2), round(d['eager_ms_per_microbatch'],2), d['launch'], d.get('graph_note'))"
done
