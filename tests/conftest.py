"""pytest configuration: the `gpu` marker (tests that need an MI355X) and import paths.

CPU tests (`-m "not gpu"`) cover the oracle against the reference's golden vectors, the host
logic (schema, settings, group expressions, automaton compiler, flattener) and that libkwgpu.so
loads and exports every symbol of include/kwgpu.h. GPU tests (`-m gpu`) are the parity tests:
they call the hot path through the C ABI and compare with the oracle.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "policy-server_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
