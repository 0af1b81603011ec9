"""Instruction mix of a kernel's basic blocks from `hipcc --cuda-device-only -S` output.

  python3 tools/isa_count.py <file.s> <kernel-name-substring> [top]

Prints the kernel's VALU / MAD / SALU / memory instruction counts and its `top`
largest basic blocks (a hot loop body is usually the largest block), so that an
A/B of a field-arithmetic change can be read as instructions per addition
before it is timed on the GPU.
"""
import re
import sys


def kernels(text):
    for m in re.finditer(r"^(_Z\S+):\s*(;.*)?$", text, re.M):
        start = m.end()
        end = text.find(".Lfunc_end", start)
        if end > start:
            yield m.group(1), text[start:end]


def mix(lines):
    v = [l for l in lines if l.startswith("v_")]
    return {
        "instr": len(lines),
        "valu": len(v),
        "mad64": sum(l.startswith("v_mad_u64_u32") for l in v),
        "cndmask": sum(l.startswith("v_cndmask") for l in v),
        "salu": sum(l.startswith("s_") for l in lines),
        "vmem": sum(l.startswith(("global_", "buffer_", "flat_")) for l in lines),
        "lds": sum(l.startswith("ds_") for l in lines),
    }


def main():
    path, pat = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    text = open(path).read()
    for name, body in kernels(text):
        if pat not in name:
            continue
        blocks, cur, label = [], [], "entry"
        for raw in body.split("\n"):
            l = raw.split(";")[0].strip()
            if not l or l.startswith("."):
                if l.startswith(".LBB"):
                    pass
                else:
                    continue
            if l.endswith(":"):
                blocks.append((label, cur))
                label, cur = l[:-1], []
                continue
            cur.append(l)
        blocks.append((label, cur))
        allins = [l for _, b in blocks for l in b]
        print(name, mix(allins))
        for label, b in sorted(blocks, key=lambda x: -len(x[1]))[:top]:
            print("  ", label, mix(b))


if __name__ == "__main__":
    main()
