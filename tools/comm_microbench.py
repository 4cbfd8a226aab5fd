"""Host + device cost of one small all_reduce, world size 1: torch.distributed vs
the native communicator, on the default stream and on a side stream."""
import os
import socket
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    from psx.parallel.comm import make_comm

    comm = make_comm(0, 1, dev)
    x = torch.zeros(6150, device=dev)
    n = int(os.environ.get("N", "2000"))

    def run(name, fn):
        for _ in range(20):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"{name:40s} host {1e6 * (t1 - t0) / n:8.2f} us/call  total {1e6 * (t2 - t0) / n:8.2f} us/call", flush=True)

    run("torch all_reduce", lambda: dist.all_reduce(x))
    run("torch all_reduce async+wait", lambda: dist.all_reduce(x, async_op=True).wait())
    run("native all_reduce (current stream)", lambda: comm.all_reduce(x))
    run("native all_reduce side+fork/join", lambda: (comm.fork(), comm.all_reduce(x, side=True), comm.join()))
    st = torch.cuda.Stream(dev)
    with torch.cuda.stream(st):
        comm.refresh_stream()
        run("native all_reduce (non-default stream)", lambda: comm.all_reduce(x))
        run("native side+fork/join (non-default stream)",
            lambda: (comm.fork(), comm.all_reduce(x, side=True), comm.join()))
        e = torch.cuda.Event()
        run("torch event record+wait (non-default)", lambda: (e.record(), torch.cuda.current_stream().wait_event(e)))
    comm.refresh_stream()
    run("x.add_(1) reference launch", lambda: x.add_(1.0))
    e = torch.cuda.Event()
    run("torch event record+wait (default)", lambda: (e.record(), torch.cuda.current_stream().wait_event(e)))
    comm.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
