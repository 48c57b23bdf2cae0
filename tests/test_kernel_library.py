"""The AOT kernel library (cekirdekler_amd/kernels/*.hsaco, built for gfx950
on the CPU): every kernel the library lists exists in its code object with
the arity the runtime launches it with.  A stale name would otherwise only
fail on the GPU box (hipModuleGetFunction: named symbol not found)."""
import pytest

from cekirdekler_amd.ops.library import ARITY, LIBRARY, code_object


@pytest.mark.parametrize("lib", sorted(LIBRARY))
def test_library_kernels_exist(lib):
    # the bundle's gfx950 ELF names every kernel's descriptor "<name>.kd" in
    # its string table
    with open(code_object(lib), "rb") as f:
        blob = f.read()
    missing = [k for k in LIBRARY[lib] if b"\0" + k.encode() + b".kd\0" not in blob]
    assert not missing, f"{lib}: not in the code object: {missing}"
    for k in LIBRARY[lib]:
        assert k in ARITY, k


def test_removed_kernel_is_detected():
    with open(code_object("sgemm_bf16"), "rb") as f:
        blob = f.read()
    assert b"\0cek_sgemm_bf16_256x256pb_sy.kd\0" not in blob  # retired in round 4
    assert b"\0cek_sgemm_bf16_256x256pb_sw.kd\0" in blob
