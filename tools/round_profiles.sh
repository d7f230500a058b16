# Round-end measurement set: bench line, rocprof kernel stats of the bench,
# PMC HBM traffic (FETCH_SIZE, WRITE_SIZE in separate passes) of the Krum
# Gram kernel at the bench shape.  Outputs under gpurun_out/.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_full.log 2>&1 || { tail -20 gpurun_out/bench_full.log; exit 1; }
tail -1 gpurun_out/bench_full.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pb -o b -- python3 /root/repo/bench.py --steps 3 --warmup 1 --no-cpu-baseline > /root/repo/gpurun_out/prof_bench.log 2>&1 || exit $?
cd /root/repo && python3 tools/rocpd_stats.py /tmp/pb/b_results.db > gpurun_out/prof_bench_stats.txt || exit $?
ls /tmp/pb >> gpurun_out/prof_bench.log
cp /tmp/pb/*stats*.csv gpurun_out/ 2>/dev/null
for C in FETCH_SIZE WRITE_SIZE; do
  K=128 P=11800394 timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d /tmp/pmc_$C -o p -- python3 tools/pairwise_only.py > gpurun_out/pmc_$C.log 2>&1 || exit $?
  python3 tools/pmc_stats.py /tmp/pmc_$C/p_results.db > gpurun_out/pmc_gram_$C.txt 2>&1
  head -4 gpurun_out/pmc_gram_$C.txt
done
python3 - <<'PY'
import json, re
def val(path):
    for line in open(path):
        if "gram_partials_kernel" in line:
            return float(line.split()[-2])
f = val("gpurun_out/pmc_gram_FETCH_SIZE.txt"); w = val("gpurun_out/pmc_gram_WRITE_SIZE.txt")
json.dump({"kernel": "gram_partials_kernel", "K": 128, "P": 11800394, "fetch_kib": f, "write_kib": w,
           "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), tools/pairwise_only.py K=128 P=11800394"},
          open("gpurun_out/gram_traffic.json", "w"), indent=1)
print("traffic GB per launch:", (2 * f + w) * 1024 / 1e9)
PY
