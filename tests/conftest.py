"""pytest configuration: the `gpu` marker and import paths.

CPU suite:  python -m pytest tests/ -x -q -m "not gpu"
GPU suite:  python -m pytest tests/ -x -q -m gpu      (MI355X box)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "image-webp_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); runs the product library")
