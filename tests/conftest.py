"""Shared test setup: paths, the `gpu` marker, native builds, fixtures.

CPU tests (-m "not gpu") check the oracle against the golden vectors, the host-side resolver
and loader against the oracle, and that libcrdt_hip.so loads and exports every C-ABI symbol.
GPU tests (-m gpu) are the parity tests proper: device merges through the C ABI vs the oracle.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

TESTS = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(TESTS)
PKG = os.path.join(ROOT, "crdt-benches_amd")
for p in (TESTS, PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

TRACES = ["automerge-paper", "rustcode", "sveltecomponent", "seph-blog1"]


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    # build the native pieces in-tree if a previous build() has not (make is incremental)
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    if not os.path.exists(os.path.join(PKG, "libcrdt_hip.so")):
        subprocess.run(["make", "-s", "-j8", "-C", PKG, "libcrdt_hip.so"], check=True)


@pytest.fixture(scope="session")
def oracle():
    from oracle_bind import Oracle
    return Oracle()


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(TESTS, "golden", "traces.json")) as f:
        return json.load(f)


_TRACE_CACHE: dict = {}


@pytest.fixture(scope="session")
def py_trace():
    from oracle_bind import load_trace

    def get(name):
        if name not in _TRACE_CACHE:
            _TRACE_CACHE[name] = load_trace(name)
        return _TRACE_CACHE[name]
    return get


@pytest.fixture(scope="session")
def ctx():
    import crdt_hip
    c = crdt_hip.Context(0)
    yield c
    c.close()


def trace_path(name: str) -> str:
    return os.path.join(ROOT, "traces", f"{name}.json.gz")
