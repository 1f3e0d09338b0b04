# Top-level convenience targets.
.PHONY: all lib test test-gpu spec-test-bls spec-test-bls-oracle bench clean

all: lib

lib:
	$(MAKE) -C lambda_ethereum_consensus_amd/csrc -j16

# README.md:106-110 of the reference documents `make spec-test-bls`; here it runs every
# BLS data.yaml (committed fixtures + consensus-spec-tests vectors if dropped into
# tests/vectors) through the GPU engine with the reference runner's pass rules.
spec-test-bls: lib
	python3 tests/spec_runner.py tests/golden/bls $(wildcard tests/vectors)

spec-test-bls-oracle:
	python3 tests/spec_runner.py --oracle tests/golden/bls $(wildcard tests/vectors)

test:
	python3 -m pytest tests -q -m "not gpu"

test-gpu: lib
	python3 -m pytest tests -q -m gpu

bench: lib
	python3 bench.py

clean:
	$(MAKE) -C lambda_ethereum_consensus_amd/csrc clean
