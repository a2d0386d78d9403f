import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through librbx.so on cuda:0)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def client():
    """One engine context for the GPU tests (fails loudly if librbx.so is missing)."""
    from redisson_amd import RedissonClient

    c = RedissonClient(0)
    yield c
    c.shutdown()


@pytest.fixture
def fresh(client):
    """Per-test name prefix (the keyspace is shared inside the session context)."""
    import uuid

    return "t" + uuid.uuid4().hex[:10]
