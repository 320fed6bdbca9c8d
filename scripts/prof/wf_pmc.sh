# PMC counters of one fused Winograd launch shape (scripts/prof/wf_one.py), three passes within the per-block slot limits
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/wpmc1 -o run -- python3 scripts/prof/wf_one.py > gpurun_out/wpmc1.log 2>&1 || { tail -5 gpurun_out/wpmc1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/wpmc2 -o run -- python3 scripts/prof/wf_one.py > gpurun_out/wpmc2.log 2>&1 || { tail -5 gpurun_out/wpmc2.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --output-format csv -d gpurun_out/wpmc3 -o run -- python3 scripts/prof/wf_one.py > gpurun_out/wpmc3.log 2>&1 || { tail -5 gpurun_out/wpmc3.log; echo pass3 failed; }
for d in wpmc1 wpmc2 wpmc3; do f=$(find gpurun_out/$d -name "*counter_collection.csv" | head -1); [ -n "$f" ] && python3 - "$f" <<'PY'
import csv, sys, collections
rows = [r for r in csv.DictReader(open(sys.argv[1])) if 'wino_fused' in r.get('Kernel_Name', '')]
agg = collections.defaultdict(float); n = collections.defaultdict(set)
for r in rows:
    agg[r['Counter_Name']] += float(r['Counter_Value']); n[r['Counter_Name']].add(r['Dispatch_Id'])
for k in sorted(agg): print(f"{k:32s} {agg[k] / max(1, len(n[k])):.4g} per dispatch ({len(n[k])} dispatches)")
PY
done
