"""The C-ABI library loads on a CPU-only host and exports every entry point include/sdhip.h declares;
the ctypes descriptor layout matches the C struct (checked by compiling the header with gcc)."""
import ctypes
import os
import re
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "sdhip.h")


def _declared():
    text = re.sub(r"/\*.*?\*/", " ", open(HEADER).read(), flags=re.S)
    return sorted(set(re.findall(r"\bint\s+(sd_\w+)\s*\(", text)))


def test_library_exports_all_declared_symbols():
    from sdreamer import _native as nat
    names = _declared()
    assert len(names) >= 40
    missing = [n for n in names if not hasattr(nat.lib, n)]
    assert not missing, missing
    assert sorted(nat.exported_symbols()) == names
    assert nat.ABI_VERSION == 1


def test_gemm_desc_layout_matches_c():
    from sdreamer import _native as nat
    src = '#include <stdio.h>\n#include <stddef.h>\n#include "sdhip.h"\nint main(void){printf("%zu %zu %zu %zu",' \
          ' sizeof(sd_gemm_desc), offsetof(sd_gemm_desc, M), offsetof(sd_gemm_desc, ksplit),' \
          ' offsetof(sd_gemm_desc, beta)); return 0;}\n'
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "t")
        subprocess.run(["gcc", "-I", os.path.dirname(HEADER), c, "-o", exe], check=True)
        out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split()
    G = nat.GemmDesc
    assert [int(x) for x in out] == [ctypes.sizeof(G), G.M.offset, G.ksplit.offset, G.beta.offset]


@pytest.mark.parametrize("cname,pyname,probe", [
    ("sd_rssm_scan", "ScanDesc", ["B", "eps", "seed", "seed_ptr", "group_offset", "W0", "WlT", "reset", "stoch", "dl",
                                  "work", "ld_g2", "row_tile", "trace", "trace_slot"]),
    ("sd_imagine", "ImagineDesc", ["eps", "seed", "seed_ptr", "row_offset", "Wa", "Wao", "Wl", "feats", "work",
                                   "t_end", "actor_h0"]),
    ("sd_stat_req", "StatReq", ["x", "n", "kind", "out", "scale"]),
    ("sd_stats", "Stats", ["r", "nreq"]),
])
def test_struct_layout_matches_c(cname, pyname, probe):
    from sdreamer import _native as nat
    S = getattr(nat, pyname)
    fmt = " ".join(["%zu"] * (len(probe) + 1))
    args = ", ".join([f"sizeof({cname})"] + [f"offsetof({cname}, {f})" for f in probe])
    src = f'#include <stdio.h>\n#include <stddef.h>\n#include "sdhip.h"\nint main(void){{printf("{fmt}", {args}); return 0;}}\n'
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "t")
        subprocess.run(["gcc", "-I", os.path.dirname(HEADER), c, "-o", exe], check=True)
        out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split()
    assert [int(x) for x in out] == [ctypes.sizeof(S)] + [getattr(S, f).offset for f in probe]


def test_kernels_refuse_cpu_tensors():
    import torch
    from sdreamer import kernels as K
    with pytest.raises(TypeError):
        K.gemm(torch.zeros(2, 2), torch.zeros(2, 2), torch.zeros(2, 2))


def test_dreamer_refuses_cpu_device():
    import copy
    from sdreamer.config import load_config
    from sdreamer.dreamer import Dreamer

    class Sp:
        shape = (6,)

    class Spaces:
        spaces = {"image": type("S", (), {"shape": (64, 64, 3)})()}
    cfg = load_config("dmc/cnn", ["device=cpu"])
    with pytest.raises(RuntimeError):
        Dreamer(copy.deepcopy(cfg.model), Spaces(), Sp())
