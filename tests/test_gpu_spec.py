"""GPU: every golden BLS fixture through the HIP engine (the `make spec-test-bls` gate)."""
import os

import pytest

from tests import spec_runner

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "bls")
VECTORS = os.path.join(os.path.dirname(__file__), "vectors")  # consensus-spec-tests, when present


@pytest.fixture(scope="module")
def gbls():
    from lambda_ethereum_consensus_amd import bls

    return bls


def test_golden_fixtures_on_gpu(gbls):
    res = spec_runner.run_dir(gbls, GOLDEN)
    assert len(res) >= 80
    bad = [(h, os.path.basename(d), det) for h, d, ok, det in res if not ok]
    assert not bad, bad


def test_golden_outcomes_identical_to_oracle(gbls):
    """Stronger than the runner's pass rule: the exact ({:ok,_}|{:error,msg}) outcome."""
    from oracle import bls12_381 as o

    for handler, case_dir in spec_runner.discover(GOLDEN):
        inp, _ = spec_runner.load_case(case_dir)
        args = {
            "sign": lambda m: (inp["privkey"], inp["message"]),
            "verify": lambda m: (inp["pubkey"], inp["message"], inp["signature"]),
            "aggregate": lambda m: (inp,),
            "eth_aggregate_pubkeys": lambda m: (inp,),
            "fast_aggregate_verify": lambda m: (inp["pubkeys"], inp["message"], inp["signature"]),
            "eth_fast_aggregate_verify": lambda m: (inp["pubkeys"], inp["message"], inp["signature"]),
            "aggregate_verify": lambda m: (inp["pubkeys"], inp["messages"], inp["signature"]),
        }[handler](None)
        got = getattr(gbls, handler)(*args)
        exp = getattr(o, handler)(*args)
        assert got == exp, (handler, os.path.basename(case_dir), got, exp)


@pytest.mark.skipif(not os.path.isdir(VECTORS), reason="consensus-spec-tests vectors not present (no network)")
def test_consensus_spec_vectors(gbls):
    res = spec_runner.run_dir(gbls, VECTORS)
    bad = [(h, d) for h, d, ok, _ in res if not ok]
    assert not bad, bad
