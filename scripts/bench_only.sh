cd /root/repo
timeout -k 10 300 python bench.py --no-cpu --steps 5 > gpurun_out/bench_exp.json 2> gpurun_out/bench_exp.err || { tail -20 gpurun_out/bench_exp.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/bench_exp.json')); r=d['roofline']
print({k:(round(v['avg_launch_ms'],3), round(v['frac'],3)) for k,v in r['kernels'].items()})"
