# Build tools/probe/gj_probe (the generated gj_rows extracted from fr_coop.hip)
set -e
cd "$(dirname "$0")"
python3 - <<'PY'
s = open("../../assistedmanipulation_amd/csrc/fr_coop.hip").read()
a = s.index("#ifdef GJ_EXEC_NOP")
b = s.index("\n}\n", s.index("void gj_rows")) + 3
open("gj_rows_gen.inc", "w").write(s[a:b])
PY
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 $1 gj_probe.hip -o gj_probe
