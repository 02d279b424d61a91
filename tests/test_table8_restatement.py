"""CPU side of the Table-8 pipeline tests (tests/test_gpu_table8.py): its numpy restatement of
get_rand_list (GPU_Runtime Test.cu:52-78, words laid out as four rows of N) agrees with the
oracle's row-major gather (Oracle.sample_problems), so the GPU tests' two checkers describe
the same selection."""
import numpy as np

from conftest import load_golden
from test_gpu_table8 import _restated_rand_list


def test_restated_get_rand_list_equals_oracle_gather(oracle):
    g = load_golden("cpp_wall.npz")
    ps32, pt32 = g["pool_src"], g["pool_tar"]
    rng = np.random.default_rng(5)
    n = 10_007
    words = rng.integers(0, 2**32 - 1, size=(4, n), dtype=np.uint32, endpoint=True)
    words[:, :3] = [[0, 0xFFFFFFFF, ps32.shape[0]]] * 4
    d_src, d_tar = _restated_rand_list(words, ps32.astype(np.float64), pt32.astype(np.float64))
    # the oracle gathers rows of 4 indices: hypothesis id's row is column id of the word list
    s, t = oracle.sample_problems(ps32, pt32, np.ascontiguousarray(words.T))
    assert np.array_equal(d_src.T, s.astype(np.float64))
    assert np.array_equal(d_tar.T, t.astype(np.float64))
