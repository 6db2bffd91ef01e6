"""Check that no instruction touches the destination VGPRs of an inline-asm global_load
between the load and the next inline-asm s_waitcnt (the asm loads are invisible to the
compiler's hazard tracking).  Usage: check_asm_loads.py kernel.s [symbol-prefix]"""
import re
import sys

RANGE = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(text):
    out = set()
    for a, b, c in RANGE.findall(text):
        if c:
            out.add(int(c))
        else:
            out.update(range(int(a), int(b) + 1))
    return out


def main():
    lines = open(sys.argv[1]).read().splitlines()
    pref = sys.argv[2] if len(sys.argv) > 2 else ""
    inside = not pref
    bad = 0
    checked = 0
    i = 0
    while i < len(lines):
        ln = lines[i]
        if pref and ln.startswith(pref):
            inside = True
        if inside and ln.strip() == "s_endpgm" and pref:
            inside = False
        m = re.match(r"\s*global_load_dwordx4 (v\[\d+:\d+\]),", ln)
        if inside and m and i > 0 and "ASMSTART" in lines[i - 1]:
            dst = regs(m.group(1))
            checked += 1
            j = i + 1
            while j < len(lines):
                t = lines[j].split(";")[0]
                if "s_waitcnt vmcnt" in t and "ASMSTART" in lines[j - 1]:
                    break
                if t.strip() and not t.strip().startswith(".") and regs(t) & dst:
                    if not re.match(r"\s*global_load_dwordx4 ", t):  # a second asm load into other regs
                        print("line %d: %s touches %s (load at %d)" % (j + 1, t.strip(), m.group(1), i + 1))
                        bad += 1
                j += 1
        i += 1
    print("asm loads checked: %d, violations: %d" % (checked, bad))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
