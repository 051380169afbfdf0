"""GPU: data-parallel ``fit`` from a partitioned Kafka topic through ``Autoencoder._fit_stream_dp``
(2 ranks rehearsed on GPU 0, SML_SHARE_GPU0=1: gloo + same-device IPC), each rank streaming
its own offset ranges of the 8 partitions through the native C++ feed.  Same checks as the CPU
test (tests/test_stream_dp.py): shares disjoint and complete, every filtered row trained once
per epoch, equal step counts, bit-identical replicas -- on the persistent kernel with the
in-kernel P2P exchange (batch 100, cardata-v3's job), on the throughput engine and on the
launch path."""
import pytest

from test_stream_dp import check_run, make_broker, run_ranks

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def broker(cuda_device):
    b = make_broker(rows=60013, partitions=8, failure_rate=0.02)
    yield b
    b.stop()


@pytest.mark.parametrize("engine,batch,dp,want", [
    ("persistent", 100, "auto", "persistent+p2p"),
    ("throughput", 4096, "rccl", "throughput"),
    ("launch", 256, "rccl", "launch"),
])
def test_fit_stream_dp_gpu(tmp_path, broker, engine, batch, dp, want):
    ranks = run_ranks(tmp_path, broker, 2, batch=batch, epochs=2, device="cuda", assign="split", native="1",
                      engine=engine, dp=dp, extra_env={"SML_SHARE_GPU0": "1"}, timeout=300)
    assert all(str(z["engine"]) == want for z in ranks), [str(z["engine"]) for z in ranks]
    check_run(broker, ranks, batch, 2)
