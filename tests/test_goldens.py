"""Reference unit-test goldens, carried verbatim:
load_balance (reference tests/load_balance.py), partition_{grad,inv}_ranks
(tests/worker_allocator.py), get_block_boundary (tests/block_divide.py)."""
import pytest

from distributed_kfac_pytorch_amd.utils import (load_balance, partition_grad_ranks,
                                                partition_inv_ranks, get_block_boundary,
                                                WorkerAllocator)


@pytest.mark.parametrize('n, work, expected', [
    (1, [1], [0]),
    (1, [1, 2], [0, 0]),
    (2, [1, 2], [1, 0]),
    (2, [1, 1, 2], [1, 1, 0]),
    (2, [1, 1, 1, 1], [0, 1, 0, 1]),
    (3, [1, 1, 1, 1], [0, 1, 2, 0]),
    (3, [5, 8, 5, 12, 5, 7, 6], [1, 1, 0, 0, 1, 2, 2]),
])
def test_load_balance(n, work, expected):
    assert load_balance(n, work) == expected


def test_load_balance_errors():
    with pytest.raises(ValueError):
        load_balance(1, [])
    with pytest.raises(ValueError):
        load_balance(0, [1])


def test_partition_grad_ranks():
    assert partition_grad_ranks(16, 8) == [[0, 8], [1, 9], [2, 10], [3, 11], [4, 12], [5, 13],
                                           [6, 14], [7, 15]]
    assert partition_grad_ranks(16, 2) == [[0, 2, 4, 6, 8, 10, 12, 14], [1, 3, 5, 7, 9, 11, 13, 15]]
    assert partition_grad_ranks(8, 8) == [[0], [1], [2], [3], [4], [5], [6], [7]]
    assert partition_grad_ranks(8, 5) == [[0, 5], [1, 6], [2, 7], [3], [4]]
    assert partition_grad_ranks(8, 4) == [[0, 4], [1, 5], [2, 6], [3, 7]]
    assert partition_grad_ranks(8, 3) == [[0, 3, 6], [1, 4, 7], [2, 5]]
    assert partition_grad_ranks(8, 2) == [[0, 2, 4, 6], [1, 3, 5, 7]]
    assert partition_grad_ranks(8, 1) == [[0, 1, 2, 3, 4, 5, 6, 7]]
    assert partition_grad_ranks(2, 1) == [[0, 1]]
    assert partition_grad_ranks(2, 2) == [[0], [1]]
    assert partition_grad_ranks(1, 1) == [[0]]


def test_partition_inv_ranks():
    assert partition_inv_ranks(16, 8) == [[0, 1, 2, 3, 4, 5, 6, 7], [8, 9, 10, 11, 12, 13, 14, 15]]
    assert partition_inv_ranks(8, 8) == [[0, 1, 2, 3, 4, 5, 6, 7]]
    assert partition_inv_ranks(8, 5) == [[0, 1, 2, 3, 4], [5, 6, 7]]
    assert partition_inv_ranks(8, 4) == [[0, 1, 2, 3], [4, 5, 6, 7]]
    assert partition_inv_ranks(8, 3) == [[0, 1, 2], [3, 4, 5], [6, 7]]
    assert partition_inv_ranks(8, 2) == [[0, 1], [2, 3], [4, 5], [6, 7]]
    assert partition_inv_ranks(8, 1) == [[0], [1], [2], [3], [4], [5], [6], [7]]
    assert partition_inv_ranks(2, 1) == [[0], [1]]
    assert partition_inv_ranks(2, 2) == [[0, 1]]
    assert partition_inv_ranks(1, 1) == [[0]]


@pytest.mark.parametrize('index, count, shape, start, end', [
    (0, 1, [100, 100], [0, 0], [100, 100]),
    (0, 2, [100, 100], [0, 0], [50, 50]),
    (1, 2, [100, 100], [50, 50], [100, 100]),
    (0, 3, [100, 100], [0, 0], [33, 33]),
    (1, 3, [100, 100], [33, 33], [66, 66]),
    (2, 3, [100, 100], [66, 66], [100, 100]),
    (0, 1, [1, 1], [0, 0], [1, 1]),
    (42, 100, [100, 100], [42, 42], [43, 43]),
    (42, 100, [100, 1000], [42, 420], [43, 430]),
])
def test_block_boundary(index, count, shape, start, end):
    assert get_block_boundary(index, count, shape) == (start, end)


def test_block_boundary_errors():
    with pytest.raises(ValueError):
        get_block_boundary(100, 100, [100, 1000])
    with pytest.raises(ValueError):
        get_block_boundary(1, 100, [10, 10])


def test_worker_allocator_layout_hybrid():
    """8 ranks, HYBRID 0.25 -> inverse groups of 2, strided gradient groups."""
    alloc = WorkerAllocator(8, 0.25, group_factory=lambda r: tuple(r))
    assert alloc.bcast_inv_ranks == [[0, 1], [2, 3], [4, 5], [6, 7]]
    assert alloc.bcast_grad_ranks == [[0, 2, 4, 6], [1, 3, 5, 7]]
    src = alloc.get_inv_ranks(5)
    assert src == [4, 5]
    pairs = alloc.get_grad_groups(src)
    assert [p[0] for p in pairs] == [4, 5, 4, 5, 4, 5, 4, 5]
    with pytest.raises(ValueError):
        WorkerAllocator(8, 3 / 8.0, group_factory=lambda r: r)
