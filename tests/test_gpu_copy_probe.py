"""The bench's copy-ceiling probe (bench.py measure_copy, cpk_stream.hip copy_kernel /
copy_lds_kernel) copies exactly, in every form the sweep times: register and LDS-DMA staging,
default and non-temporal access, grid-strided and contiguous shares, grids that leave a partial
round of chunks (the plain-copy tail).  Not the codec: the roofline's reference point."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu



@pytest.fixture(scope="module")
def codec():
    import capnproto_amd

    c = capnproto_amd.Codec(0)
    yield c
    c.close()


FORMS = (0, 1, 2, 4, 5, 6, 8, 9, 10, 12, 13, 14, 16, 17, 18, 20, 21, 22)


@pytest.mark.parametrize("nbytes", [(8 << 20) + 48, 3 << 20])
def test_copy_forms_exact(codec, nbytes):
    torch = codec.torch
    rng = np.random.default_rng(nbytes)
    src = torch.from_numpy(rng.integers(0, 256, nbytes, dtype=np.uint8)).to(codec.device)
    s = torch.cuda.current_stream(codec.device)
    for form in FORMS:
        for g in (7, 1024, 4096):
            dst = torch.zeros_like(src)
            st = codec.lib.cpk_debug_copy(C.c_void_p(dst.data_ptr()), C.c_void_p(src.data_ptr()),
                                          nbytes, (form << 24) | g, C.c_void_p(s.cuda_stream))
            assert st == 0
            torch.cuda.synchronize()
            assert torch.equal(dst, src), (form, g)
