#!/bin/bash
# tests + default bench + per-kernel A/B of VARIANTS on CFGS + unpack step counters (var_diag.so)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out; PWD_R=$(pwd)
TAG=${1:-r04f}
# (variants that are not built are skipped; SPLIT defaults on)
# (tools/ab_variants.txt, if present, adds variants to VARIANTS)
[ -f tools/ab_variants.txt ] && VARIANTS="${VARIANTS:-base} $(cat tools/ab_variants.txt)"
V=""; for v in ${VARIANTS:-base}; do if [ $v = base ] || [ -f capnproto_amd/var_$v.so ]; then V="$V $v"; fi; done
export VARIANTS="$V"; SPLIT=${SPLIT-1}
bash tools/gpu_ab3.sh $TAG || exit 1
# GPU tests with each variant library in TESTVARS swapped in
cp capnproto_amd/libcpk_hip.so /tmp/cpk_main.so
for v in $TESTVARS; do
  cp capnproto_amd/var_$v.so capnproto_amd/libcpk_hip.so
  timeout -k 10 400 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests_$v.log 2>&1
  rc=$?; echo "== tests $v"; tail -2 gpurun_out/${TAG}_tests_$v.log
  cp /tmp/cpk_main.so capnproto_amd/libcpk_hip.so
  [ $rc = 0 ] || [ $rc = 1 ] || exit 1
done
for f in capnproto_amd/var_diag*.so; do
  [ -f $f ] || continue
  n=$(basename $f .so)
  timeout -k 10 300 python3 tools/diag_unpack.py $f ${DIAG_CFGS:-c2 c3 c4 split} > gpurun_out/${TAG}_$n.log 2>&1
  rc=$?; echo "== $n"; grep -v amdgpu.ids gpurun_out/${TAG}_$n.log | tail -4; [ $rc = 0 ] || exit 1
done
if [ -n "$SPLIT" ]; then
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD_R/gpurun_out/${TAG}_split" -o run \
    -- python3 "$PWD_R/tools/split_prof.py" > "$PWD_R/gpurun_out/${TAG}_split.log" 2>&1) || { echo "split prof failed"; tail -5 gpurun_out/${TAG}_split.log; exit 1; }
  tail -3 gpurun_out/${TAG}_split.log
  python3 - gpurun_out/${TAG}_split <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/*kernel_stats.csv")[0]
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))[:8]:
    print(r["Name"].split("(")[0][-40:], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
fi
if [ -n "$SMALL" ]; then
  for zc in default 0; do
  if [ $zc = default ]; then unset CPK_HOST_ZERO_COPY; else export CPK_HOST_ZERO_COPY=$zc; fi
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$PWD_R/gpurun_out/${TAG}_small_$zc" -o run \
    -- python3 "$PWD_R/tools/small_prof.py" 100 > "$PWD_R/gpurun_out/${TAG}_small_$zc.log" 2>&1) || { echo "small prof failed"; tail -5 gpurun_out/${TAG}_small_$zc.log; exit 1; }
  echo "== small zero-copy=$zc"; grep "message_bytes" gpurun_out/${TAG}_small_$zc.log
  python3 - gpurun_out/${TAG}_small_$zc <<'PY'
import csv, glob, sys
ev = []
for f in glob.glob(sys.argv[1] + "/*kernel_trace.csv") + glob.glob(sys.argv[1] + "/*memory_copy_trace.csv"):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name") or r.get("Direction") or "copy"
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name.split("(")[0][-30:]))
ev.sort()
prev = None
for s, e, n in ev[-12:]:
    gap = (s - prev) / 1e3 if prev else 0.0
    print(f"  {n:32s} dur {(e - s) / 1e3:7.1f} us  gap {gap:7.1f} us")
    prev = e
PY
  done
  unset CPK_HOST_ZERO_COPY
fi
