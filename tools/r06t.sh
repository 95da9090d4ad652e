set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/$1
run() { tag=$1; envs=$2; shift 2
  env $envs timeout -k 10 300 python -u bench.py --tp-proxy 8 --steps 5 "$@" > $O.$tag.json 2> $O.$tag.err || { echo $tag failed; tail -5 $O.$tag.err; exit 1; }
  python -c "import json; d=json.load(open('$O.$tag.json')); print('$tag', round(d['value']), round(d['ms_per_microbatch'],2), round(d['eager_ms_per_microbatch'],2))"
}
run new A=0
run old "PICOTRON_ROPE_FUSE_MIN_TILES=96 PICOTRON_SWIGLU_FUSE_MIN_TILES=192"
run new_mix0 PICOTRON_GEMM_MIX=0
run new_swb512 PICOTRON_SWIGLU_BWD_MIN_TILES=512
run new2 A=0
run new_mb4 A=0 --mbs 4
run old_mb4 "PICOTRON_ROPE_FUSE_MIN_TILES=96 PICOTRON_SWIGLU_FUSE_MIN_TILES=192" --mbs 4
