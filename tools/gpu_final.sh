#!/bin/bash
# Round-end call with a candidate kernel change: GPU tests with the candidate library
# (capnproto_amd/var_t.so, built from alt_src/), a per-kernel A/B against the in-tree library, the
# faster correct one installed (sources too, so kernel_source_hash matches what is measured), then
# the PMC traffic passes (C2, C4, C3) copied into profiles/ and the round evidence (gpu_round.sh).
#   gpurun --timeout 1180 -- bash tools/gpu_final.sh TAG
set -o pipefail
TAG=${1:-r03e}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
choice=base
if [ -f capnproto_amd/var_t.so ]; then
  cp capnproto_amd/libcpk_hip.so /tmp/cpk_main.so
  cp capnproto_amd/var_t.so capnproto_amd/libcpk_hip.so
  ok=1
  timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_cand_tests.log 2>&1 || ok=0
  tail -2 gpurun_out/${TAG}_cand_tests.log
  cp /tmp/cpk_main.so capnproto_amd/libcpk_hip.so
  if [ $ok = 1 ]; then
    VARIANTS="t base" CFGS="c4 c2" bash tools/gpu_prof_ab.sh ${TAG}_ab > gpurun_out/${TAG}_ab.txt 2>&1 || { cat gpurun_out/${TAG}_ab.txt; exit 1; }
    cat gpurun_out/${TAG}_ab.txt
    choice=$(python3 - "$R/gpurun_out" "${TAG}_ab" <<'PY'
import csv, glob, sys
def t(v, c):
    f = glob.glob(f"{sys.argv[1]}/{sys.argv[2]}_{v}_{c}/*kernel_stats.csv")[0]
    return sum(float(r["AverageNs"]) for r in csv.DictReader(open(f)) if "pack_tile" in r["Name"])
new = t("t", "c4") + 20 * t("t", "c2")
old = t("base", "c4") + 20 * t("base", "c2")
print("t" if new < 0.98 * old else "base")
PY
)
  fi
fi
echo "chosen: $choice"
if [ "$choice" = t ]; then
  cp alt_src/* capnproto_amd/csrc/
  cp capnproto_amd/var_t.so capnproto_amd/libcpk_hip.so
fi
echo "$choice" > gpurun_out/${TAG}_choice.txt
for c in c2 c4 c3; do
  bash tools/gpu_pmc3.sh ${TAG}_$c $c > gpurun_out/${TAG}_pmc_$c.out 2>&1 || { echo "pmc $c failed"; tail -5 gpurun_out/${TAG}_pmc_$c.out; exit 1; }
  cp gpurun_out/${TAG}_${c}_traffic_$c.json profiles/traffic_$c.json
done
echo "pmc done"
bash tools/gpu_round.sh $TAG
