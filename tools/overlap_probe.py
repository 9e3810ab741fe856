"""Co-scheduling probe: the posterior scan (latency-bound, <=128 workgroups per launch) alone vs concurrently with
encoder convolutions on another stream, with and without stream priorities. Decides whether pipelining the encoder
against the scan can pay."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "safe-dreamer_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    from sdreamer.config import load_config
    from sdreamer.dreamer import Dreamer
    cfg = load_config("dmc/cnn", ["device=cuda:0", "model.compile=False"])
    torch.manual_seed(0)
    ag = Dreamer(cfg.model, bench._Spaces({"image": bench._Sp((64, 64, 3))}), bench._Sp((6,)))
    B, T = 16, 64
    g = torch.Generator().manual_seed(0)
    img = (torch.randint(0, 256, (B, T, 64, 64, 3), generator=g, dtype=torch.uint8).float() / 255).cuda()
    act = (torch.rand(B, T, 6, generator=g) * 2 - 1).cuda()
    first = torch.zeros(B, T, dtype=torch.bool, device="cuda")
    first[:, 0] = True
    init = (torch.zeros(B, 32, 16, device="cuda"), torch.zeros(B, 2048, device="cuda"))
    with torch.no_grad():
        embed = ag.encoder({"image": img})

    def scan():
        with torch.no_grad():
            ag.rssm.observe(embed, act, init, first, seed=1)

    def enc_work(n=3):
        with torch.no_grad():
            for _ in range(n):
                ag.encoder({"image": img})

    def timed(fn, stream):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(stream):
            s.record()
            fn()
            e.record()
        return s, e

    for prio in (0, -1):
        main = torch.cuda.Stream(priority=prio)
        other = torch.cuda.Stream(priority=0)
        for _ in range(2):
            scan()
        torch.cuda.synchronize()
        s, e = timed(scan, main)
        torch.cuda.synchronize()
        alone = s.elapsed_time(e)
        so, eo = timed(enc_work, other)
        s, e = timed(scan, main)
        torch.cuda.synchronize()
        print(f"priority {prio}: scan alone {alone:.3f} ms, scan beside encoder {s.elapsed_time(e):.3f} ms, "
              f"encoder x3 {so.elapsed_time(eo):.3f} ms", flush=True)
    so, eo = timed(enc_work, torch.cuda.current_stream())
    torch.cuda.synchronize()
    print(f"encoder x3 alone {so.elapsed_time(eo):.3f} ms")
    # CU-masked encoder stream (hipExtStreamCreateWithCUMask): keep every k-th CU free for the scan
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    for keep_every in (8, 2, -8):
        bits = [0] * ((ncu + 31) // 32)
        for cu in range(ncu):
            use = (cu % 8 == 0) if keep_every < 0 else (cu % keep_every != 0)  # -8: encoder on 1/8 of the CUs
            if use:
                bits[cu // 32] |= 1 << (cu % 32)
        arr = (ctypes.c_uint32 * len(bits))(*bits)
        h = ctypes.c_void_p()
        rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(len(bits)), arr)
        other = torch.cuda.ExternalStream(h.value)
        scan_s = torch.cuda.Stream()
        so, eo = timed(enc_work, other)
        torch.cuda.synchronize()
        alone = so.elapsed_time(eo)
        so, eo = timed(enc_work, other)
        s, e = timed(scan, scan_s)
        torch.cuda.synchronize()
        used = sum(bin(b).count("1") for b in bits)
        print(f"cu mask rc={rc}: encoder on {used} CUs: x3 alone {alone:.3f} ms; scan beside "
              f"{s.elapsed_time(e):.3f} ms, encoder x3 beside {so.elapsed_time(eo):.3f} ms", flush=True)


if __name__ == "__main__":
    main()
