"""Page-level check of a codec host-memory history (IGGY_CODEC_HOSTMEM_LOG): every
registration whose page span meets a live registration's page span, with the test that
made it. Diagnostic only.

usage: python scripts/hostmem_pages.py <hostmem.log>
"""
import re
import sys


def main(path):
    live, test, hits, n_reg = {}, None, [], 0
    for ln in open(path):
        p = ln.split()
        if len(p) > 2 and p[1] == "test":
            test = p[3]
            continue
        m = re.search(r"hostmem: (.*) \[(0x[0-9a-f]+), (0x[0-9a-f]+)\) (\d+) B", ln)
        if not m:
            continue
        what, a, b = m.group(1), int(m.group(2), 16), int(m.group(3), 16)
        if what == "register":
            n_reg += 1
            pa, pb = a & ~4095, (b + 4095) & ~4095
            for k, (qa, qb, t) in live.items():
                if pa < qb and qa < pb:
                    hits.append((test, a, b, k, t))
            live[a] = (pa, pb, test)
        elif what.startswith("unregister"):
            live.pop(a, None)
    print(f"{path}: {n_reg} registrations, {len(hits)} sharing a page with a live registration, "
          f"{len(live)} live at the end")
    for t, a, b, k, tk in hits:
        print(f"  {t}: [{a:#x}, {b:#x}) shares a page with the range at {k:#x} ({tk})")


if __name__ == "__main__":
    main(sys.argv[1])
