"""PCIe copy issue pattern probe: does a stream of 8 MiB host-to-device
copies run back to back, or does each pay a start-up gap?  Pinned host
memory, one GPU; SDMA both ways (torch's copy_ with non_blocking).

    python tools/h2d_chunks_probe.py [out.json]

Cases (256 MiB up, optionally 256 MiB down at the same time):
  one_copy        one 256 MiB copy
  chunks_32       32 x 8 MiB on one stream
  chunks_32_ev    the same with an event recorded after every second copy
                  (the event pipeline records one per blob)
  chunks_16x16    16 MiB chunks
  two_streams_32  the 32 chunks alternating between two streams (two SDMA queues)
  duplex_32       chunks_32 up while 32 x 8 MiB go down on another stream
  down_*          downloads: one copy, chunks on one stream, chunks alternating
                  over two streams (256 MiB, and the Mandelbrot image's 64 MiB)
"""
import json
import sys
import time

import torch

MB = 1 << 20
N = 256 * MB


def timed(fn, reps=5):
    best = 1e30
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t) * 1e3)
    return round(best, 3)


def main():
    host = torch.empty(N, dtype=torch.uint8).pin_memory()
    host_dn = torch.empty(N, dtype=torch.uint8).pin_memory()
    dev = torch.empty(N, dtype=torch.uint8, device="cuda")
    dev_dn = torch.empty(N, dtype=torch.uint8, device="cuda")
    up, dn = torch.cuda.Stream(), torch.cuda.Stream()
    evs = [torch.cuda.Event() for _ in range(64)]

    def chunks(size, ev=False):
        k = N // size
        with torch.cuda.stream(up):
            for i in range(k):
                dev[i * size:(i + 1) * size].copy_(host[i * size:(i + 1) * size], non_blocking=True)
                if ev and i % 2 == 1:
                    evs[i // 2].record(up)

    up2 = torch.cuda.Stream()

    def two_streams(size):
        k = N // size
        for i in range(k):
            with torch.cuda.stream(up if i % 2 == 0 else up2):
                dev[i * size:(i + 1) * size].copy_(host[i * size:(i + 1) * size], non_blocking=True)

    def duplex():
        with torch.cuda.stream(dn):
            for i in range(32):
                host_dn[i * 8 * MB:(i + 1) * 8 * MB].copy_(dev_dn[i * 8 * MB:(i + 1) * 8 * MB], non_blocking=True)
        chunks(8 * MB)

    res = {"one_copy_ms": timed(lambda: chunks(N)),
           "chunks_32_ms": timed(lambda: chunks(8 * MB)),
           "chunks_32_ev_ms": timed(lambda: chunks(8 * MB, True)),
           "chunks_16x16_ms": timed(lambda: chunks(16 * MB)),
           "two_streams_32_ms": timed(lambda: two_streams(8 * MB)),
           "duplex_32_ms": timed(duplex),
           "down_alone_32_ms": timed(lambda: [host_dn[i * 8 * MB:(i + 1) * 8 * MB].copy_(
               dev_dn[i * 8 * MB:(i + 1) * 8 * MB], non_blocking=True) for i in range(32)])}
    # downloads: the whole 256 MiB, and the Mandelbrot image's 64 MiB in one
    # copy, 8 chunks on one stream, 8 chunks alternating over two streams
    dn2 = torch.cuda.Stream()

    def down(total, size, streams):
        k = total // size
        for i in range(k):
            with torch.cuda.stream(streams[i % len(streams)]):
                host_dn[i * size:(i + 1) * size].copy_(dev_dn[i * size:(i + 1) * size], non_blocking=True)

    res["down_one_copy_ms"] = timed(lambda: down(N, N, [dn]))
    res["down_two_streams_32_ms"] = timed(lambda: down(N, 8 * MB, [dn, dn2]))
    res["down64_one_copy_ms"] = timed(lambda: down(64 * MB, 64 * MB, [dn]))
    res["down64_8_chunks_ms"] = timed(lambda: down(64 * MB, 8 * MB, [dn]))
    res["down64_8_chunks_two_streams_ms"] = timed(lambda: down(64 * MB, 8 * MB, [dn, dn2]))
    res["down64_16_chunks_two_streams_ms"] = timed(lambda: down(64 * MB, 4 * MB, [dn, dn2]))
    res["one_copy_gbps"] = round(N / res["one_copy_ms"] / 1e6, 1)
    res["chunks_32_gbps"] = round(N / res["chunks_32_ms"] / 1e6, 1)
    js = json.dumps(res)
    print(js)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            f.write(js + "\n")


if __name__ == "__main__":
    main()
