"""CPU-side checks of the C-ABI library: it loads, exports every declared symbol,
and its host-side orientation table equals the reference's (no GPU compute here)."""
import ctypes
import os
import re

import pytest

from reinforcementlearning_blokus_amd import _native as N
from tests.conftest import ROOT, load_golden


def declared_symbols():
    text = open(os.path.join(ROOT, "include", "blokus_hip.h")).read()
    return sorted(set(re.findall(r"^(?:int|const char\s*\*|void\s*\*)\s*(bk_\w+)\s*\(", text, flags=re.M)))


def test_header_and_binding_agree():
    assert declared_symbols() == sorted(N.EXPORTS)


def test_library_exports_every_symbol():
    lib = N.load()
    for name in declared_symbols():
        assert hasattr(lib, name), name
    assert lib.bk_abi_version() == N.ABI_VERSION == 7
    assert lib.bk_tables_version() >= 1


def test_struct_sizes():
    assert ctypes.sizeof(N.BkState) == 256
    assert ctypes.sizeof(N.BkResult) == 32
    assert ctypes.sizeof(N.BkRolloutCfg) == 40


def test_orientation_table_matches_reference():
    ref = load_golden("pieces.json")
    tab = N.orient_table()
    assert len(tab) == 91
    for (pid, o, offs), r in zip(tab, ref):
        assert (pid, o) == (r["piece_id"], r["orientation"])
        assert [list(x) for x in offs] == r["offsets"]


def test_invalid_arguments_rejected_without_gpu():
    lib = N.load()
    assert lib.bk_destroy(None) == N.EINVAL
    assert lib.bk_orient_info(91, None, None, None, None) == N.EINVAL
    assert lib.bk_set_tuning(None, 0, 1) == N.EINVAL
    assert lib.bk_get_tuning(None, 0, None) == N.EINVAL
    assert lib.bk_mcts_set_done(None, None) == N.EINVAL
    assert lib.bk_host_free(None) == N.OK


def test_environment_read_only_at_handle_creation():
    """the library reads its BK_* tuning variables once, in bk_create
    (into the handle; bk_set_tuning changes them), never inside an entry point -- a stray
    variable cannot change a running caller's kernel choice.  Checked on the source: the
    only getenv calls sit in bk_create."""
    src = open(os.path.join(ROOT, "reinforcementlearning_blokus_amd", "csrc", "blokus_kernels.hip")).read()
    create = src.index("int bk_create(")
    create_end = src.index("\nint bk_destroy(", create)
    calls = [m.start() for m in re.finditer(r"\bgetenv\s*\(", src)]
    assert calls and all(create < c < create_end for c in calls), calls
    # the header's tuning keys and the binding's names agree, in order
    hdr = open(os.path.join(ROOT, "include", "blokus_hip.h")).read()
    keys = re.findall(r"^\s*BK_TUNE_(\w+)\s*(?:=\s*0)?,", hdr, flags=re.M)
    assert ["BK_" + k for k in keys] == list(N.TUNE_KEYS), keys
    names = re.findall(r'"(BK_\w+)"', src[src.index("kTuneNames"):src.index("};", src.index("kTuneNames"))])
    assert names == list(N.TUNE_KEYS)


def test_gpu_free_container_fails_loudly():
    """With no GPU, creating a handle raises instead of falling back."""
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except ImportError:
        pass
    with pytest.raises(N.NativeUnavailable):
        N.Handle(0)


def test_one_hip_runtime_per_process():
    """_native.load() imports torch first, so the library binds torch's libamdhip64 (same
    soname) instead of pulling in /opt/rocm's as a second runtime (two runtimes in one
    process leave torch without a GPU; tools/runtime_order_probe.py).  Checked in a
    fresh interpreter from the process's memory map; no GPU call is made."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from reinforcementlearning_blokus_amd import _native as N\n"
            "N.load()\n"
            "libs = sorted({l.split()[-1] for l in open('/proc/self/maps') if 'libamdhip64' in l})\n"
            "print(len(libs)); print(libs)\n") % ROOT
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    n = int(out.stdout.splitlines()[0])
    assert n == 1, out.stdout
