set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/profiles
export TMPDIR=/tmp
WORKLOADS="coffee 16 coffee;coffee 16 coffee_noms --no-multiscattering;lamp 16 lamp" bash tools/refresh_profiles.sh || exit $?
cp gpurun_out/profiles/r04_*_pmc_traffic.json profiles/
: > gpurun_out/profiles/r04_configs.jsonl
for item in "cornell" "coffee" "coffee --no-multiscattering" "spaceship" "spaceship_close" "lamp"; do
  timeout -k 10 400 python bench.py --config $item --steps 16 --warmup 2 --no-cpu-baseline --repeats 3 --roofline-images 16 --spaceship-spp 0 > gpurun_out/cfg.json 2>gpurun_out/cfg.err || exit $?
  tail -1 gpurun_out/cfg.json >> gpurun_out/profiles/r04_configs.jsonl
  python -c "import json;d=json.load(open('gpurun_out/cfg.json'));print('$item', d['ms_per_spp'], d['repeat_ms_per_spp'], d['value'], d['roofline'].get('frac'), d.get('pipeline_roofline',{}).get('frac'), d['roofline'].get('frac_algorithmic'), d['material']['avg_launch_us'])"
done
