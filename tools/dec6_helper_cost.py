"""Static instruction counts of rc_decompress_dec6s's helper loop (rc_slot.h
slot_help_iter), per pass type, from the kernel's assembly:
  idle: no new packet, no chunk to load, nothing to announce
  busy: a chunk loaded, stored to the slot and announced
usage: python tools/dec6_helper_cost.py dec6.s   (hipcc --cuda-device-only -S of rc_dec6.hip)
Used with a -DDEC6_HELP_COUNT build's pass counts (ws.counters[5..6]) to
split the kernel's PMC instruction counts between helper and decoding waves."""
import re
import sys

lines = [l.rstrip("\n") for l in open(sys.argv[1])]
sleep = max(i for i, l in enumerate(lines) if re.match(r"\s*s_sleep ", l))
# the helper loop: from its header block (the one holding the m_ctl / m_pkt reads) to the back branch
body = []
for l in lines[: sleep + 4]:
    s = l.strip()
    if not s or s.startswith(";"):
        continue
    body.append(s)
# blocks by label
blocks, cur = {}, None
for s in body:
    m = re.match(r"(\.LBB\d+_\d+):", s)
    if m:
        cur = m.group(1)
        blocks[cur] = []
        continue
    if cur:
        blocks[cur].append(s.split()[0])
# the loop header: the last block before the sleep that starts with two ds_read_b32
labels = list(blocks)
head = [b for b in labels if blocks[b][:2] == ["ds_read_b32", "ds_read_b32"]][-1]
order = labels[labels.index(head):]


def kind(op):
    # (as the SQ_INSTS_* counters split them: branches and SMEM apart from SALU;
    # waits, nops and sleeps in none of them)
    if op.startswith("v_"):
        return "valu"
    if op.startswith(("s_waitcnt", "s_nop", "s_sleep", "s_setprio", "s_endpgm")):
        return "wait"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("global_") or op.startswith("buffer_") or op.startswith("flat_"):
        return "vmem"
    return "other"


def count(ops):
    c = {}
    for op in ops:
        k = kind(op)
        c[k] = c.get(k, 0) + 1
    return c


def upto(b, pred):
    """ops of block b up to and including the first op matching pred"""
    out = []
    for op in blocks[b]:
        out.append(op)
        if pred(op):
            break
    return out


br = lambda op: op.startswith("s_cbranch")  # noqa: E731
# blocks: 0 header (m reads, the leave store), 1 new packet, 2 join, 3 inq, 4 the chunk load,
# 5 its wait (a partial chunk's byte loop in 6-7 when a lane has one), 8 slot store, 9 check sum,
# 10 h_ctl store, 11 fin / sleep / back branch
b = [blocks[x] for x in order]
idle = upto(order[0], br) + b[3] + upto(order[4], lambda o: o == "s_cbranch_vccz") + upto(order[10], br) + b[11]
busy = upto(order[0], br) + b[3] + b[4] + upto(order[5], br) + b[8] + b[9] + b[10] + b[11]
for name, ops in (("idle", idle), ("busy", busy)):
    c = count(ops)
    print(name, len(ops), c)
print("blocks:", [(x, len(blocks[x])) for x in order])
