"""Audit the replay kernel ISA: the reserved registers that receive the
inline-asm prefetch loads (v112..v127, kNhBase in replay.hip; v152..v167,
kNhBaseGen, in replay_gen_kernel and replay_inl_kernel) must be referenced only by inline asm (the prefetch loads and the wait+copy reads),
anywhere in the kernel.  Usage: python tools/check_nh_regs.py build/asm/replay-...-gfx950.s"""
import re
import sys


def regs_of(s):
    out = set()
    for m in re.finditer(r"v\[(\d+):(\d+)\]", s):
        out |= set(range(int(m.group(1)), int(m.group(2)) + 1))
    for m in re.finditer(r"\bv(\d+)\b", s):
        out.add(int(m.group(1)))
    return out


def audit(path):
    return (audit_one(path, "_ZN6fognet12_GLOBAL__N_113replay_kernelILi", 112)
            + audit_one(path, "_ZN6fognet12_GLOBAL__N_117replay_gen_kernelILi", 152)
            + audit_one(path, "_ZN6fognet12_GLOBAL__N_117replay_inl_kernelILi", 152))


def audit_one(path, kernel_prefix, base):
    text = open(path).read().split("\n")
    bad_total = 0
    found = 0
    for npl, pol in [(n, p) for n in (1, 2, 4) for p in (1, 16)]:  # policies REF_V3, EXT_LAT
        name = f"{kernel_prefix}{npl}ELi{pol}EEEvNS_10ReplayArgsE"
        starts = [i for i, ln in enumerate(text) if ln.startswith(f"{name}:")]
        if not starts:
            continue
        found += 1
        s = starts[0]
        body = []
        for ln in text[s + 1:]:
            if ln.startswith(".Lfunc_end"):
                break
            body.append(ln.strip())
        nh = set()
        in_asm = False
        for ln in body:
            if ln.startswith(";;#ASMSTART"):
                in_asm = True
            elif ln.startswith(";;#ASMEND"):
                in_asm = False
            elif in_asm and ln.startswith("global_load_dwordx4"):
                nh |= regs_of(ln.split(",")[0])
        assert nh and min(nh) >= base and max(nh) < base + 16, f"prefetch destinations outside the reserved range: {sorted(nh)}"
        bad = []
        in_asm = False
        for ln in body:
            if ln.startswith(";;#ASMSTART"):
                in_asm = True
                continue
            if ln.startswith(";;#ASMEND"):
                in_asm = False
                continue
            if not ln or ln.startswith(";") or ln.startswith("."):
                continue
            if not in_asm and regs_of(ln) & nh:
                bad.append(ln)
        print(f"{kernel_prefix[26:-3]} NPL={npl} policy={pol}: prefetch registers {sorted(nh)}; compiler references outside asm: {len(bad)}")
        for b in bad[:20]:
            print("   ", b)
        bad_total += len(bad)
    assert found == 6, f"expected 6 {kernel_prefix} instantiations in the ISA, found {found}"
    return bad_total


if __name__ == "__main__":
    sys.exit(1 if audit(sys.argv[1]) else 0)
