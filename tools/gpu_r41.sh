# configs[2]: forest predict_proba over 20M then 100M resident rows (bit-exact vs sklearn).
set -u
mkdir -p gpurun_out
timeout -k 10 200 python -u bench_forest.py --rows 20000000 > gpurun_out/forest20m_r41.json 2> gpurun_out/forest20m_r41.err \
    || { tail -20 gpurun_out/forest20m_r41.err; exit 1; }
cat gpurun_out/forest20m_r41.json
timeout -k 10 300 python -u bench_forest.py > gpurun_out/forest100m_r41.json 2> gpurun_out/forest100m_r41.err \
    || { tail -20 gpurun_out/forest100m_r41.err; exit 1; }
cat gpurun_out/forest100m_r41.json
