# SQ activity of config 5's small memory-side kernels (one counter pass, kernel regex), per kernel name.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
RX='layernorm|lora_proj|geglu|nf4_dequant|lora_wgrad'
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "$RX" --output-format csv -d $O/pmc -o p -- python3 -u $R/bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc.log 2>&1
python3 - $O <<'PY'
import csv, glob, sys, collections
rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + "/pmc/**/*counter_collection.csv", recursive=True)[0])))
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    k = r["Kernel_Name"].split("(")[0].split("<")[0][-40:]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in acc.items():
    w = c["SQ_WAVE_CYCLES"] or 1
    print(f"{k:40s} valu_active {c['SQ_ACTIVE_INST_VALU'] / w:.3f}  wait_inst {c['SQ_WAIT_INST_ANY'] / w:.3f}  "
          f"wait_any {c['SQ_WAIT_ANY'] / w:.3f}  active_any {c['SQ_ACTIVE_INST_ANY'] / w:.3f}")
PY
