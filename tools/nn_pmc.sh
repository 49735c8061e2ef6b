#!/bin/bash
# PMC passes over the network-only microbenchmark (tools/nn_bench.py).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/nnpmc
i=0
for set in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" "SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $set -d gpurun_out/nnpmc/p$i -o p --output-format csv -- python tools/nn_bench.py --iters 5 > gpurun_out/nnpmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/nnpmc/p$i.log; exit 1; }
done
python - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(list)
for f in glob.glob("gpurun_out/nnpmc/p*/p_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "kNNForward" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print("%-28s %14.1f" % (k, sum(v) / len(v)))
PY
