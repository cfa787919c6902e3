"""Per-conv roofline of the ResNet-50 b256 forward from a rocprofv3 kernel trace: maps the
forward conv dispatches of the last full step to the layers (torchvision order) and prints
time vs max(FLOP / 2.5 PF/s, compulsory bytes / 6 TB/s)."""
import csv
import sys


def layers(N=256):
    out = [("stem7x7", N, 224, 3, 64, 7, 2)]
    H, cin = 56, 64
    for stage, (w, nb) in enumerate([(64, 3), (128, 4), (256, 6), (512, 3)]):
        for b in range(nb):
            s = 2 if (b == 0 and stage > 0) else 1
            out.append((f"l{stage+1}.{b}.c1", N, H, cin, w, 1, 1))
            if b == 0:  # the block computes its identity right after c1 (models/resnet.py)
                out.append((f"l{stage+1}.{b}.ds", N, H, cin, 4 * w, 1, s))
            out.append((f"l{stage+1}.{b}.c2", N, H, w, w, 3, s))
            Ho = H // s
            out.append((f"l{stage+1}.{b}.c3", N, Ho, w, 4 * w, 1, 1))
            cin, H = 4 * w, Ho
    return out


def main(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    opt = [i for i, r in enumerate(rows) if "adamw_mt_k<1" in r["Kernel_Name"]]
    sel = rows[opt[-2] + 1: opt[-1] + 1]
    fw = [r for r in sel if "conv_fwd_k" in r["Kernel_Name"] and ", true, false, false, 1, 0, 4, 0" in r["Kernel_Name"]]
    L = layers()
    tot_t = tot_r = 0.0
    print(f"{'layer':12s} {'us':>7s} {'roof_us':>7s} {'eff':>5s} {'TF/s':>6s} {'TB/s':>5s}")
    for (name, N, H, C, K, R, s), r in zip(L, fw):
        P = (H + 2 * (R // 2) - R) // s + 1
        fl = 2.0 * N * P * P * K * C * R * R
        by = 2.0 * (N * H * H * C + N * P * P * K)
        t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        roof = max(fl / 2.5e15, by / 6e12) * 1e6
        tot_t += t
        tot_r += roof
        print(f"{name:12s} {t:7.1f} {roof:7.1f} {roof / t:5.2f} {fl / t / 1e6:6.0f} {by / t / 1e6:5.2f}")
    print(f"forward convs: {len(fw)} dispatches, {tot_t / 1e3:.3f} ms vs roofline {tot_r / 1e3:.3f} ms")


if __name__ == "__main__":
    main(sys.argv[1])
