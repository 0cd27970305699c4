"""Transcribe the reference's state-machine known-answer tables into fixture files.

Run once in the build container (the reference tree is not present on the GPU box):

    python tests/golden/extract_kats.py /root/reference/src/state_machine.zig

Each `try check(<table>)` block of a test in the in-scope range (create_accounts, linked chains,
create_transfers, two-phase, expiry, chain rollback, balancing, and the
get_account_transfers / get_account_balances queries: state_machine.zig:2767-3571) is
written verbatim as data to tests/golden/kat_<test-name>[_<k>].tbl, with a header naming the
source lines. The rows are inputs and expected outputs only (events, expected result codes,
expected balances); they are parsed by tests/kat.py, which mirrors testing/table.zig:8-93 and the
harness `check()` at state_machine.zig:2507-2765.
"""
import os
import re
import sys

IN_SCOPE = (2767, 3571)


def main(path):
    lines = open(path).read().split("\n")
    out_dir = os.path.dirname(os.path.abspath(__file__))
    test_name = None
    block = None
    count = {}
    written = []
    for lineno, line in enumerate(lines, start=1):
        m = re.match(r'^test "(.*)" \{', line)
        if m:
            test_name = m.group(1)
            continue
        if "try check(" in line:
            block = {"start": lineno, "rows": []}
            continue
        if block is not None:
            s = line.strip()
            if s.startswith("\\\\"):
                block["rows"].append(s[2:].rstrip())
            elif s.startswith(");"):
                block["end"] = lineno
                if IN_SCOPE[0] <= block["start"] <= IN_SCOPE[1]:
                    slug = re.sub(r"[^a-z0-9]+", "_", test_name.lower()).strip("_")
                    k = count.get(slug, 0)
                    count[slug] = k + 1
                    name = f"kat_{slug}" + (f"_{k}" if k else "") + ".tbl"
                    with open(os.path.join(out_dir, name), "w") as f:
                        f.write(f"# test \"{test_name}\" — state_machine.zig:{block['start']}-{block['end']}\n")
                        for r in block["rows"]:
                            f.write(r + "\n")
                    written.append(name)
                block = None
    print("\n".join(written))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference/src/state_machine.zig")
