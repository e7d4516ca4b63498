"""CPU checks of the drop-in boundary: libbgcn.so loads without a GPU, exports every
entry point include/bgcn.h declares, and the ctypes mirrors of the header's structs
have the C layout (sizes and field offsets measured by compiling the header with gcc)."""
import ctypes
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "bgcn.h")


def _declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^[A-Za-z_][\w \*]*?\b(bgcn_\w+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_header_declares_what_the_binding_lists():
    from bigcn_amd import _lib
    assert _declared_functions() == sorted(_lib.EXPORTED_SYMBOLS)
    assert set(_lib._SIGS) == set(_lib.EXPORTED_SYMBOLS)


def test_library_loads_and_exports_every_symbol():
    from bigcn_amd import _lib
    lib = _lib.load_library()
    for name in _declared_functions():
        assert hasattr(lib, name), name
    assert lib.bgcn_abi_version() == 12


def test_workspace_queries_without_gpu():
    from bigcn_amd import _lib
    lib = _lib.load_library()
    assert lib.bgcn_graph_workspace_size(100, 50) > 0
    assert lib.bgcn_spmm_workspace_size(150, 64) > 0
    assert lib.bgcn_bigcn_workspace_size(1000, 8, 5000, 64) > lib.bgcn_bigcn_workspace_size(100, 8, 5000, 64)
    n = lib.bgcn_train_step_workspace_size(1000, 8, 5000, 4, 990, 990)
    assert n > lib.bgcn_bigcn_workspace_size(1000, 8, 5000, 64)
    # weight images: W1^T [F][128] + W2^T [2][F+64][64] fp32 + the bf16 split images
    assert lib.bgcn_weight_images_size(5000) >= 4 * (5000 * 128 + 2 * 5064 * 64)
    assert lib.bgcn_weight_images_size(0) == 0


def test_invalid_arguments_fail_before_any_device_work():
    from bigcn_amd import _lib
    lib = _lib.load_library()
    rc = lib.bgcn_spmm(None, None, None, None, 0, 0, None, 64, None, 64, 64, None, 0, None, 0, None)
    assert rc == -1
    assert b"bad rows" in lib.bgcn_last_error()
    a = _lib.StepArgs()
    assert lib.bgcn_train_step(ctypes.addressof(a), None, 0, None) == -1
    assert lib.bgcn_adam_step(None, None) == -1


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_ctypes_struct_layout_matches_header(tmp_path):
    from bigcn_amd import _lib
    from bigcn_amd.optim import AdamArgs
    structs = {
        "bgcn_graph_view": _lib.GraphView, "bgcn_csr_out": _lib.CsrOut,
        "bgcn_bigcn_args": _lib.BiGCNArgs, "bgcn_step_args": _lib.StepArgs,
        "bgcn_adam_args": AdamArgs, "bgcn_batch": _lib.BatchDesc, "bgcn_spmm_plan": _lib.SpmmPlan,
    }
    from bigcn_amd import feed
    structs.update({"bgcn_tree_store": feed._TreeStoreArgs, "bgcn_loader_batch": feed._LoaderBatch,
                    "bgcn_loader_stats": feed._LoaderStats})
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void) {"]
    for cname, py in structs.items():
        lines.append(f'printf("{cname} sizeof %zu\\n", sizeof({cname}));')
        for fname, _ in py._fields_:
            lines.append(f'printf("{cname} {fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append("return 0; }")
    c = tmp_path / "layout.c"
    c.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c99", "-o", str(exe), str(c)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    got = {}
    for line in out:
        if line:
            s, f, v = line.split()
            got[(s, f)] = int(v)
    for cname, py in structs.items():
        assert got[(cname, "sizeof")] == ctypes.sizeof(py), cname
        for fname, _ in py._fields_:
            assert got[(cname, fname)] == getattr(py, fname).offset, (cname, fname)


def test_constants_match_header():
    import re
    from bigcn_amd import _lib
    text = open(HEADER).read()
    for name in ("BGCN_DEGREE_ON_COL", "BGCN_DEGREE_ON_ROW", "BGCN_EPI_NONE", "BGCN_EPI_RELU",
                 "BGCN_FEAT_AUTO", "BGCN_FEAT_DENSE", "BGCN_SPARSE_CAP", "BGCN_DTYPE_F32",
                 "BGCN_DTYPE_BF16"):
        m = re.search(rf"#define {name} (\d+)", text)
        assert m, name
        assert int(m.group(1)) == getattr(_lib, name), name
    from bigcn_amd import optim
    for name in ("TD_W1", "BU_W1", "TD_W2", "BU_W2"):
        m = re.search(rf"#define BGCN_IMAGE_{name} (\d+)", text)
        assert m and int(m.group(1)) == getattr(optim, "IMAGE_" + name), name
