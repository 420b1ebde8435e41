"""pytest configuration.

Markers: ``gpu`` = needs an MI355X (run with ``-m gpu`` on the GPU box); the
rest runs on CPU.  GPU tests never import torch: the C-ABI library carries its
own HIP runtime binding ("One HIP runtime per process").
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD Instinct MI355X (gfx950)")
    config.addinivalue_line("markers", "slow: long-running CPU test")
