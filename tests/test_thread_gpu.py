"""ThreadComm with GPU tensors: T host threads share one MI355X; the thread phase is the
multi-input K1 reduce kernel (NIN = T) instead of the reference's pairwise Exchanger tree."""
import threading

import pytest

torch = pytest.importorskip("torch")

from mp4x import CommUtils, Operands, Operators  # noqa: E402

pytestmark = pytest.mark.gpu


def _threads(tc, fn):
    T = tc.getThreadNum()
    out, errs = [None] * T, []

    def body(t):
        try:
            tc.setThreadId(t)
            out[t] = fn(t)
        except BaseException as e:  # noqa
            errs.append(e)
            tc._barrier.abort()

    ths = [threading.Thread(target=body, args=(t,)) for t in range(T)]
    [x.start() for x in ths]
    [x.join() for x in ths]
    if errs:
        raise errs[0]
    return out


@pytest.mark.parametrize("T", [2, 5, 11])
def test_thread_allreduce_gpu(T):
    from mp4x.launch import init_from_env
    tc = init_from_env(thread_num=T, heartbeat=False)
    n = 100_003

    def body(t):
        x = torch.full((n,), float(t + 1), device="cuda")
        tc.allreduceArray(x, Operands.FLOAT_OPERAND(), Operators.Float.SUM, 7, n - 5)
        torch.cuda.synchronize()
        assert torch.all(x[7:n - 5] == T * (T + 1) / 2) and x[0] == t + 1
        y = torch.full((n,), 1 << (t % 30), device="cuda", dtype=torch.int64)
        tc.allreduceArray(y, Operands.LONG_OPERAND(), Operators.Long.BITS_OR, 0, n)
        torch.cuda.synchronize()
        assert torch.all(y == sum(1 << (j % 30) for j in set(range(T))))
        # reduce-scatter with [1][T] counts
        f = CommUtils.createThreadArrayFroms(n, 1, T)
        to = CommUtils.createThreadArrayTos(n, 1, T)
        counts = [[to[0][j] - f[0][j] for j in range(T)]]
        z = torch.ones(n, device="cuda", dtype=torch.float64)
        tc.reduceScatterArray(z, Operands.DOUBLE_OPERAND(), Operators.Double.SUM, 0, counts)
        torch.cuda.synchronize()
        assert torch.all(z[f[0][t]:to[0][t]] == T)
        # allgather
        w = torch.full((n,), -1.0, device="cuda")
        w[f[0][t]:to[0][t]] = t
        tc.allgatherArray(w, Operands.FLOAT_OPERAND(), f, to)
        torch.cuda.synchronize()
        for j in range(T):
            assert torch.all(w[f[0][j]:to[0][j]] == j)
        return True

    assert all(_threads(tc, body))
    tc.close(0)
