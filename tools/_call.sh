set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for pass in 1 2; do
for cfg in spaceship spaceship_close coffee lamp; do
for tr in 1 0; do
  DCRT_LDS_TRIM=$tr timeout -k 10 300 python bench.py --config $cfg --steps 16 --warmup 2 --no-cpu-baseline --repeats 3 --roofline-images 2 --spaceship-spp 0 > gpurun_out/ab.json 2>gpurun_out/ab.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));r=d['roofline'];print('$cfg trim=$tr', d['ms_per_spp'], d['repeat_ms_per_spp'], 'cast us', r['avg_launch_us'], r['launch'])"
done
done
done
