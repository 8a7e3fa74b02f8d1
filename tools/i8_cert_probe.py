"""Why does the int8 single-query certificate fail on the clustered corpus?  Emulates the
K9q quantisation in torch (per-row absmax / 127, round to nearest) and prints, per
in-distribution query: the int8 bound E (screen_bound's VERIFY_BF16_Q32 form with the
shadow's maxima), tau as the sample pass sets it (8th largest per-list maximum of every
16th 32-row block; lists = 2 x 256 workgroups), the survivor count, the k-th best screen
score, the live count (screen >= cs_k - 2E) and the k-th exact score.  GPU box only."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mediquery-rag_amd"))

import torch  # noqa: E402

from mediquery_hip import synth  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    n, k = 1_000_000, 5
    rows, _ = synth.clustered_corpus_device(n, 768, dev)
    rows = torch.nn.functional.normalize(rows, dim=1)
    amax = rows.abs().amax(1, keepdim=True)
    scale = amax / 127
    r8 = torch.clamp(torch.round(rows / scale), -127, 127)
    deq = r8 * scale
    dmax = (rows - deq).norm(dim=1).max().item()
    cmax = deq.norm(dim=1).max().item()
    g = 2 * 768 * 2 ** -24
    q, _ = synth.queries_device(8, rows, seed=synth.QUERY_SEED + 11, planted_frac=1.0)
    print("dmax %.5f cmax %.5f" % (dmax, cmax))
    n_blocks = (n + 31) // 32
    G = 512
    for j in range(q.shape[0]):
        qq = q[j]
        E = (dmax + g * (cmax + dmax) + g * cmax) * 1.001 * qq.norm().item()
        exact = rows @ qq
        scr = (r8 @ qq) * scale.squeeze(1)
        # sample pass: blocks b with b % 16 == 0, list = (b / 16) % G (workgroup stride walk)
        blk = torch.arange(n, device=dev) // 32
        sel = (blk % 16) == 0
        lst = (blk[sel] // 16) % G
        lmax = torch.full((G,), -float("inf"), device=dev).scatter_reduce(0, lst, scr[sel], "amax")
        tau = torch.sort(lmax, descending=True).values[7].item()
        surv = scr >= tau
        cnt = int(surv.sum())
        cs = torch.sort(scr[surv], descending=True).values
        csk = cs[k - 1].item()
        live = int((scr[surv] >= csk - 2 * E).sum())
        ek = torch.topk(exact, k).values[-1].item()
        e64 = torch.topk(exact, 64).values[-1].item()
        print("q%d E %.4f tau %.4f count %d cs_k %.4f live %d e_k %.4f e_64 %.4f cert(tau) %s gap %.4f"
              % (j, E, tau, cnt, csk, live, ek, e64, tau + E < ek, ek - tau))


if __name__ == "__main__":
    main()
