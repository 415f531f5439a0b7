"""Box-ordered model problems (amg_par_stencil_create_boxes / amg_host_csr_stencil): the grid
cut into bx x by x bz boxes numbered box by box is P A P^T of the natural-order stencil, for
every rank's slice; boxes (1, 1, P) reproduce the z-slab generator exactly.  CPU only (host
halves of the C-ABI against the oracle's generators and permutation)."""
import numpy as np
import pytest

CASES = [("7pt", (12, 10, 9), (2, 2, 2)), ("7pt", (13, 11, 10), (3, 1, 2)), ("27pt", (9, 8, 7), (2, 2, 2)),
         ("5pt", (17, 13), (3, 2)), ("7pt", (8, 8, 8), (1, 1, 1))]


def oracle_gen(O, kind, dims):
    return {"5pt": O.gen_5pt, "7pt": O.gen_7pt, "27pt": O.gen_27pt}[kind](*dims)


@pytest.mark.parametrize("kind,dims,boxes", CASES)
@pytest.mark.parametrize("nranks", [1, 2, 3])
def test_box_order_is_permuted_stencil(oracle, kind, dims, boxes, nranks):
    from raptor_amd import box_order
    from raptor_amd.host import HostCSR

    nb = int(np.prod(boxes))
    if nranks > nb:
        pytest.skip("fewer boxes than ranks")
    O = oracle
    perm = box_order(dims, boxes)
    assert np.array_equal(np.sort(perm), np.arange(perm.size))
    B = O.permute(oracle_gen(O, kind, dims), perm).to_scipy()
    rows = 0
    for r in range(nranks):
        M = HostCSR.stencil(kind, dims, boxes, rank=r, nranks=nranks).to_scipy_local()
        f = M.shape[0]
        ref = B[rows:rows + f]
        assert np.array_equal(M.indptr, ref.indptr) and np.array_equal(M.indices, ref.indices)
        assert np.array_equal(M.data, ref.data)
        rows += f
    assert rows == B.shape[0]


@pytest.mark.parametrize("kind,dims", [("7pt", (9, 8, 12)), ("27pt", (7, 6, 9))])
def test_slab_boxes_equal_slab_generator(oracle, kind, dims):
    from raptor_amd.host import HostCSR

    O = oracle
    A = oracle_gen(O, kind, dims).to_scipy()
    for nranks in (1, 2, 3, 4):
        rows = 0
        for r in range(nranks):
            M = HostCSR.stencil(kind, dims, (1, 1, nranks), rank=r, nranks=nranks).to_scipy_local()
            ref = A[rows:rows + M.shape[0]]
            # z-slab rows: planes nz r / P .. nz (r + 1) / P, the natural numbering
            assert rows == (dims[2] * r // nranks) * dims[0] * dims[1]
            assert np.array_equal(M.indices, ref.indices) and np.array_equal(M.data, ref.data)
            rows += M.shape[0]
