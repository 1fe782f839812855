#!/bin/bash
# Regenerates tests/golden/lds_race_prefix_lnx.dis.gz: the disassembly of the GEMM + LayerNorm exchange
# kernels as built by the round-5 commit f3f892b WITHOUT its fix (the two `rp_waitcnt<..., 0>` LDS-read
# drains of lx_mainloop put back to `<..., 15>`, i.e. the untracked-fill build that failed the repeat
# tests, profiles logged in 58eceee).  Test infrastructure for tests/test_lds_race.py; needs git history.
set -e
cd "$(dirname "$0")/../.."
T=$(mktemp -d)
mkdir -p $T/repurpose_amd/csrc $T/include
for f in repurpose_amd/csrc/rp_gemm.hip repurpose_amd/csrc/rp_common.h include/rp_api.h; do git show f3f892b:$f > $T/$f; done
sed -i 's/rp_waitcnt<LX_PF, 0>();  \/\/ stage kt + 1/rp_waitcnt<LX_PF, 15>();  \/\/ stage kt + 1/; /for (int kt = LX_PFS; kt < nk; ++kt)/,/rp_raw_barrier/ s/rp_waitcnt<0, 0>()/rp_waitcnt<0, 15>()/' $T/repurpose_amd/csrc/rp_gemm.hip
grep -c "rp_waitcnt<LX_PF, 15>" $T/repurpose_amd/csrc/rp_gemm.hip
(cd $T && /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude -c repurpose_amd/csrc/rp_gemm.hip -o rp_gemm.o)
python - "$T/rp_gemm.o" <<'PY'
import gzip, sys
sys.path.insert(0, "tests")
import lds_race
text = lds_race.disassemble(sys.argv[1])
keep, on = [], False
for ln in text.splitlines():
    m = lds_race._FUNC.match(ln)
    if m:
        on = "gemm_lnx" in m.group(2)
    if on:
        keep.append(ln)
gzip.open("tests/golden/lds_race_prefix_lnx.dis.gz", "wt").write("\n".join(keep) + "\n")
print(len(keep), "lines")
PY
rm -rf $T
