set -o pipefail
mkdir -p gpurun_out
O=$PWD/gpurun_out/$1
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --cpu-tokens 0 --steps 10 > $O.new_$r.json 2>/dev/null || { echo new failed; exit 1; }
  (cd tools/ab/old && timeout -k 10 300 python -u bench.py --cpu-tokens 0 --steps 10 > $O.old_$r.json 2>/dev/null) || { echo old failed; exit 1; }
  python -c "import json; a=json.load(open('$O.new_$r.json')); b=json.load(open('$O.old_$r.json')); print('round $r new', round(a['value']), 'old', round(b['value']))"
done
