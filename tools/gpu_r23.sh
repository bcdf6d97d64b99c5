for e in 0 1; do
  if [ $e = 1 ]; then export FDX_PREP_NORAT=1; fi
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --breakdown > gpurun_out/norat$e.json 2> gpurun_out/norat$e.err || exit 1
  tail -1 gpurun_out/norat$e.err
done
