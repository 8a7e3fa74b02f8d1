"""Why does the int8 single-query certificate fail where it does?  Emulates the K9q
pipeline in torch for in-distribution queries over the clustered corpus: per-row absmax
int8 quantisation, the sample pass's per-list maxima (every 16th 8-row unit; unit u goes
to wave u mod W of the appending pass's grid, list = its workgroup), the r5 tau rule
tau = min(T8, max(Tk - 2E, T_FLOOR)), survivors s >= tau, per-row bounds E_r, L_k = the k-th
largest s - E_r, live = s + E_r >= L_k, and the certificate tau + E < e_k.  Prints one line
per query whose emulated certificate fails, with the failing condition, and the counts.
GPU box only."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mediquery-rag_amd"))

import torch  # noqa: E402

from mediquery_hip import synth  # noqa: E402


FLOOR = int(os.environ.get("FLOOR", "32"))  # the floor's rank (r5: 32; 16 before)


def main():
    dev = torch.device("cuda", 0)
    n, k, nq = 1_000_000, int(sys.argv[1]) if len(sys.argv) > 1 else 5, 100
    rows, _ = synth.clustered_corpus_device(n, 768, dev)
    rows = torch.nn.functional.normalize(rows, dim=1)
    amax = rows.abs().amax(1, keepdim=True)
    scale = amax / 127
    deq = torch.clamp(torch.round(rows / scale), -127, 127) * scale
    err = (rows - deq).norm(dim=1)
    dmax, cmax = err.max().item() * 1.001, deq.norm(dim=1).max().item() * 1.001
    g = 2 * 768 * 2 ** -24
    q, _ = synth.queries_device(nq, rows, seed=synth.QUERY_SEED + 11, planted_frac=1.0)
    G, W = 768, 768 * 4  # lists (workgroups) and waves of the scan at 256 CUs
    unit = torch.arange(n, device=dev) // 8
    sel = (unit % 16) == 0
    lst = ((unit[sel] // 16) % W) // 4  # sample unit u*16 -> wave (u mod W) -> its workgroup
    fails = {"floor": 0, "surv>1024": 0, "live>512": 0, "cert": 0}
    for j in range(nq):
        qq = q[j]
        qn = qq.norm().item()
        E = (qn * dmax + g * qn * (cmax + dmax) + g * qn * cmax) * 1.001 + 1e-7
        exact = rows @ qq
        scr = deq @ qq
        lmax = torch.full((G,), -float("inf"), device=dev).scatter_reduce(0, lst, scr[sel], "amax")
        T = torch.sort(lmax, descending=True).values
        t8, tk, t16 = T[7].item(), T[k - 1].item(), T[FLOOR - 1].item()
        tc = tk - 2.02 * E - 1e-6
        tau = min(t8, max(tc, t16))
        surv = torch.nonzero(scr >= tau).squeeze(1)
        Er = (qn * err[surv] * 1.001 + g * qn * (cmax + err[surv] * 1.001) + g * qn * cmax) * 1.001 + 1e-7
        lo, hi = scr[surv] - Er, scr[surv] + Er
        Lk = torch.sort(lo, descending=True).values[k - 1].item() if len(surv) >= k else -float("inf")
        live = int((hi >= Lk).sum())
        ek = torch.topk(exact, k).values[-1].item()
        why = None
        if len(surv) > 1024:
            why = "surv>1024"
        elif live > 512:
            why = "live>512"
        elif not tau + E < ek:
            why = "floor" if tc < t16 else "cert"
        if why:
            fails[why] += 1
            print("q%d %s: E %.4f tau %.4f (T8 %.4f Tk %.4f Tfloor %.4f) surv %d live %d e_k %.4f"
                  % (j, why, E, tau, t8, tk, t16, len(surv), live, ek))
    print("k", k, "fails", fails)


if __name__ == "__main__":
    main()
