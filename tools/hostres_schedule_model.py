"""Fluid model of the host-resident GEMM's PCIe schedule (8192³: A and B
uploaded as 16 panels of 8 MiB each, C downloaded in 1 MiB blocks of 512²
fp32 as soon as both panels of a block are on the device; compute taken as
free).  Link rates from the session-3/8 probes: 57 / 53 GB/s up / down
alone, 45.5 GB/s each when both directions run.  Prints the model's wall
time for the square-shell order (the runtime's) and for other upload
orders.  python tools/hostres_schedule_model.py"""
import itertools
P = 16            # panels per operand
PANEL = 8.0       # MiB per A or B panel
BLOCK = 1.0       # MiB per C block (512x512 fp32)
UP1, DN1, BOTH = 57.0*1.048576, 53.0*1.048576, 45.5*1.048576  # MiB/ms
def sim(order):
    # order: list of ('A', i) / ('B', j) uploads
    t = 0.0; a=set(); b=set(); dq=[]; done=set()
    up_left = [PANEL]*len(order); ui = 0; dn_rem = 0.0
    produced = 0
    while ui < len(order) or dq or dn_rem > 1e-9:
        up_active = ui < len(order)
        dn_active = dn_rem > 1e-9 or bool(dq)
        if dn_rem <= 1e-9 and dq:
            dq.pop(0); dn_rem = BLOCK
        ru = (BOTH if dn_active else UP1) if up_active else 0
        rd = (BOTH if up_active else DN1) if dn_active else 0
        # time to next event
        dt = min([up_left[ui]/ru] if up_active else [1e9]) 
        if dn_active: dt = min(dt, dn_rem/rd)
        t += dt
        if up_active:
            up_left[ui] -= ru*dt
            if up_left[ui] <= 1e-9:
                k, i = order[ui]; ui += 1
                (a if k=='A' else b).add(i)
                new = [(x,y) for x in a for y in b if (x,y) not in done]
                for blk in new: done.add(blk); dq.append(blk)
        if dn_active: dn_rem -= rd*dt
    return t
sq = []
for k in range(P): sq += [('A',k),('B',k)]
print('square shells', round(sim(sq),3))
# B first k0 panels then alternate
for k0 in (2,4,6,8):
    o = [('B',j) for j in range(k0)]
    rest_b = list(range(k0,P)); ai = 0
    o2=[]
    # interleave A panels with remaining B panels at ratio
    for i in range(P):
        o2.append(('A',i))
        if rest_b: o2.append(('B',rest_b.pop(0)))
    o2 += [('B',j) for j in rest_b]
    print('B first', k0, round(sim(o + o2),3))
# rectangular: ratio r A panels per B panel
for r in (2,3):
    o=[]; bi=0; ai=0
    while ai<P or bi<P:
        if bi<P: o.append(('B',bi)); bi+=1
        for _ in range(r):
            if ai<P: o.append(('A',ai)); ai+=1
    print('ratio', r, round(sim(o),3))
