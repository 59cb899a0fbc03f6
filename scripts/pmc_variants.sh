# SQ_INSTS_VALU / SQ_INSTS_SALU / SQ_INSTS_LDS / SQ_INSTS_VMEM_RD per wave of the forest kernels for several
# kernel-library variants (x2_* sensitivity builds: a phase's instruction count = variant - cur)
#   VARIANTS="cur x2_eval" gpurun -- bash scripts/pmc_variants.sh
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
L=cs230_distributed_machine_learning_amd/lib
for v in ${VARIANTS}; do
  if [ "$v" = cur ]; then lib=$L/libdml_hip.so; else lib=$L/libdml_hip_$v.so; fi
  DML_HIP_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/pmcv_$v -o p -- python3 scripts/gbench_forest.py 1000000 100 100 5 > gpurun_out/pmcv_$v.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, collections, os
for v in os.environ["VARIANTS"].split():
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    with open(f"gpurun_out/pmcv_{v}/p_counter_collection.csv") as f:
        for r in csv.DictReader(f):
            k = r["Kernel_Name"].split("(")[0][-26:]
            if "dml::" not in r["Kernel_Name"]: continue
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, d in sorted(agg.items(), key=lambda kv: -kv[1]["SQ_WAVE_CYCLES"])[:4]:
        w = d["SQ_WAVES"] or 1
        print(f"{v:10s} {k:26s} valu {d['SQ_INSTS_VALU']/w:7.0f} salu {d['SQ_INSTS_SALU']/w:7.0f} lds {d['SQ_INSTS_LDS']/w:6.0f} "
              f"vmem_rd {d['SQ_INSTS_VMEM_RD']/w:6.0f} vmem_wr {d['SQ_INSTS_VMEM_WR']/w:5.0f} cyc {4*d['SQ_WAVE_CYCLES']/w:8.0f} valu_act {d['SQ_ACTIVE_INST_VALU']/d['SQ_WAVE_CYCLES']:.3f}")
PY
