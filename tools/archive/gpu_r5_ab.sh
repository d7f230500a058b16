#!/bin/bash
# A/B of the reference-exact chain kernel's chunk size and ring depth (same box),
# then one PMC pass on the default library
set -o pipefail
mkdir -p gpurun_out/r5ab
timeout -k 10 60 ./tools/hip/valu_lat > gpurun_out/r5ab/valu_lat.txt 2>&1 || { echo "valu_lat failed"; cat gpurun_out/r5ab/valu_lat.txt; exit 1; }
cat gpurun_out/r5ab/valu_lat.txt
for v in default ref_cs64_ns4 ref_cs32_ns8 ref_cs64_ns6 ref_cs64_ns8; do
  if [ $v = default ]; then L=multimodal-fl-security_amd/lib/libflr.so; else L=abl/$v/libflr.so; fi
  FLR_LIB=$L timeout -k 10 120 python -u tools/ref_bench.py --reps 5 --check 16 > gpurun_out/r5ab/$v.json 2> gpurun_out/r5ab/$v.err || { echo "$v failed"; tail -5 gpurun_out/r5ab/$v.err; exit 1; }
  echo "$v $(cat gpurun_out/r5ab/$v.json)"
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS -d gpurun_out/r5ab/pmca -o a --output-format csv -- python3 -u tools/ref_bench.py --reps 1 --check 0 > gpurun_out/r5ab/pmca.log 2>&1 || { echo "pmc a failed"; tail -5 gpurun_out/r5ab/pmca.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d gpurun_out/r5ab/pmcb -o b --output-format csv -- python3 -u tools/ref_bench.py --reps 1 --check 0 > gpurun_out/r5ab/pmcb.log 2>&1 || { echo "pmc b failed"; tail -5 gpurun_out/r5ab/pmcb.log; exit 1; }
echo done
