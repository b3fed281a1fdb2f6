import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: multi-process / longer tests")


@pytest.fixture(scope="session")
def native_ext():
    """Build (incrementally) and import the native extension; CPU-safe."""
    import build_native
    build_native.ensure_built()
    from pytorch_distributed_tutorials_amd.ops import _ext
    return _ext.native()


@pytest.fixture(scope="session")
def gpu(native_ext):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def parse_results(text: str) -> list:
    """Every JSON object printed after a "RESULT " marker.  Ranks of a multi-process test print
    through one pipe and their lines can interleave (two payloads on one line), so each payload is
    decoded with raw_decode from its marker instead of assuming one object per line."""
    import json
    dec, res, pos = json.JSONDecoder(), [], 0
    while True:
        pos = text.find("RESULT ", pos)
        if pos < 0:
            return res
        try:
            obj, end = dec.raw_decode(text, pos + len("RESULT "))
            res.append(obj)
            pos = end
        except json.JSONDecodeError:
            pos += len("RESULT ")


def free_port() -> int:
    """A TCP port on 127.0.0.1 that is free right now (for launcher rendezvous in tests)."""
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(autouse=True)
def _keepalive(request):
    """GPU tests that compile library kernels on a fresh box (MIOpen for the stock-model
    yardsticks) can run a minute without printing; a daemon thread writes a progress mark to the
    real stderr (past pytest's capture) every 30 s so a runner's no-output watchdog sees a live
    process."""
    if request.node.get_closest_marker("gpu") is None:
        yield
        return
    import threading
    stop = threading.Event()

    def beat():
        while not stop.wait(30.0):
            try:
                sys.__stderr__.write(f"[keepalive] {request.node.name} still running\n")
                sys.__stderr__.flush()
            except Exception:
                return

    t = threading.Thread(target=beat, daemon=True)
    t.start()
    try:
        yield
    finally:
        stop.set()


@pytest.fixture(autouse=True)
def _stock_convs_without_miopen(request):
    """Stock-PyTorch yardstick models in GPU tests run their convolutions without MIOpen
    (PyTorch's own im2col + BLAS path).  On a fresh box MIOpen compiles every new conv shape
    inside the conv call while holding the GIL -- minutes for a ResNet-50 in fp32 and bf16,
    train and eval -- so no output (not even the keepalive thread's) appears meanwhile.  The
    yardsticks only need correct fp32 / bf16 convolutions, not MIOpen's."""
    if request.node.get_closest_marker("gpu") is None:
        yield
        return
    import torch
    with torch.backends.cudnn.flags(enabled=False):
        yield
