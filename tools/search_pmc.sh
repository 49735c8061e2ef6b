#!/bin/bash
# PMC passes over a short bench run; per-kernel averages for the search kernels.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/spmc
i=0
for set in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" "SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set -d gpurun_out/spmc/p$i -o p --output-format csv -- python bench.py --steps 2 --warmup 1 --rounds-per-step 50 --no-cpu-baseline --no-npz > gpurun_out/spmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/spmc/p$i.log; exit 1; }
done
python - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/spmc/p*/p_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        for tag in ("kSelect", "kBackup", "kNNForward", "kCommit"):
            if tag in k:
                agg[tag][r["Counter_Name"]].append(float(r["Counter_Value"]))
for tag, d in agg.items():
    print(tag)
    for c, v in sorted(d.items()):
        print("  %-26s %16.1f" % (c, sum(v) / len(v)))
PY
