set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/$1
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --cpu-tokens 0 > $O.probe_$r.json 2> $O.probe_$r.err || { echo bench failed; tail -5 $O.probe_$r.err; exit 1; }
  timeout -k 10 300 python -u bench.py --cpu-tokens 0 --no-probe > $O.noprobe_$r.json 2> $O.noprobe_$r.err || { echo bench failed; tail -5 $O.noprobe_$r.err; exit 1; }
  python -c "import json; a=json.load(open('$O.probe_$r.json')); b=json.load(open('$O.noprobe_$r.json')); print('round $r probe', round(a['value']), round(a['ms_per_step'],2), 'no-probe', round(b['value']), round(b['ms_per_step'],2))"
done
