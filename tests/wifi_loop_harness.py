"""The closed-loop Wi-Fi tests' MAC stand-in, run on the oracle (nsref_wifil_run, which restates it in
C++) and on the device PHY attached to the host runtime (nsgpu.Sim + wifi.LoopPhy, the closures below).

The stand-in (nsref.h: nsref_wifil_mac): at setup, Schedule (first[i], attempt i) for every phy in order,
then Simulator::Stop (stop_ts).  attempt i: if phy i's WifiPhyStateHelper state is IDLE, SendPacket and
Schedule (period, attempt i); otherwise Schedule (backoff[i], attempt i).  The m_random draw of every
EndReceive (yans-wifi-phy.cc:783) is made here, on both runs' records, with one fixed sequence per phy."""
import numpy as np

import nsref
import wifi


def scenario(n_side=4, spacing=100.0, seed=1, period=20_000_000, stop_ns=200_000_000, size=200,
             mode=wifi.DSSS_1M, preamble=wifi.PREAMBLE_LONG, dbm=16.0206 + 1.0, **phy_kw):
    x, y, z = wifi.grid(n_side, spacing)
    phys = wifi.LoopPhys(x, y, z, **phy_kw)
    rng = np.random.default_rng(seed)
    n = phys.n_phy
    first = rng.integers(0, period // 2, n).astype(np.uint64)
    backoff = (100_000 + 37_000 * np.arange(n)).astype(np.uint64)
    return dict(phys=phys, first=first, backoff=backoff, period=period, stop_ns=stop_ns, size=size, mode=mode,
                preamble=preamble, dbm=dbm)


def run_oracle(sc, log_cap=1 << 20, uid_first=0):
    ph = sc["phys"]
    cfg = ph.c_struct()
    log, ends, phys, tot = nsref.wifil_run(cfg, sc["first"], sc["backoff"], sc["period"], sc["stop_ns"], sc["size"],
                                           sc["mode"], sc["preamble"], sc["dbm"], ph.n_phy, wifi.WIFIL_END_DTYPE,
                                           wifi.PHY_COUNTERS_DTYPE, log_cap, uid_first=uid_first,
                                           reply_delay=sc.get("reply_delay"))
    return log, ends, phys, tot


def run_gpu(sc, log_cap=1 << 20, uid_first=0, listen=None, bounds=None, part=None, comm=None):
    """uid_first: m_uid before the setup calls (nsgpu_sim_set_next_uid; 0: the reference's 4).
    sc["reply_delay"] (ns, optional): the EndReceive hand-back (nsgpu_sim_wifi_set_end_handler) — at each EndReceive
    that is not cancelled and whose draw (0.5) exceeds its per, the MAC stand-in schedules a reply of that phy
    (nsref.h: nsref_wifil_mac.reply_on).  listen: the phys handed back (default: every phy when replying)."""
    import nsgpu
    ph = sc["phys"]
    sim = nsgpu.Sim()
    if uid_first:
        sim.set_next_uid(uid_first)
    lp = wifi.LoopPhy(ph, bounds=bounds, part=part, comm=comm)
    sim.attach_wifi(lp)
    sim.set_log(log_cap)
    cnt = {"sends": 0, "busy": 0, "handbacks": 0}
    txs = []  # (ts, closure uid, phy) per SendPacket: the MonitorSnifferTx records

    def attempt(i, reply=False):
        st, _ = sim.wifi_state(i)
        if st != wifi.IDLE:
            cnt["busy"] += 1
            if not reply:
                sim.schedule(int(sc["backoff"][i]), lambda: attempt(i))
            return
        txs.append((sim.now(), sim.current_uid(), i))
        sim.wifi_send(i, sc["size"], sc["dbm"], sc["mode"], sc["preamble"])
        cnt["sends"] += 1
        if not reply:
            sim.schedule(sc["period"], lambda: attempt(i))

    rd = sc.get("reply_delay")
    if rd is not None:
        def end_receive(e):  # YansWifiPhy::EndReceive's host part: the draw, then the MAC's receive callback
            cnt["handbacks"] += 1
            assert sim.now() == int(e["ts"]) and sim.current_uid() == int(e["uid"])
            if 0.5 > e["per"]:
                i = int(e["phy"])
                sim.schedule(rd, lambda: attempt(i, True))
        sim.wifi_set_end_handler(end_receive)
        for i in (range(ph.n_phy) if listen is None else listen):
            sim.wifi_listen(i)

    for i in range(ph.n_phy):
        sim.schedule(int(sc["first"][i]), (lambda i=i: lambda: attempt(i))())
    sim.stop(sc["stop_ns"])
    sim.run()
    _n, _c, digest = sim.host_stats()
    k = min(sim.dispatched(), log_cap)
    log = (sim.log[0][:k].copy(), sim.log[1][:k].copy(), sim.log[2][:k].copy())
    ends = lp.read_ends()
    phys = lp.read_phys()
    tot = dict(dispatched=sim.dispatched(), digest=digest, next_uid=sim.next_uid(), final_ts=sim.now(), **cnt)
    tot["txs"] = np.array(txs, np.uint64).reshape(-1, 3)
    lp_keep = (sim, lp)
    return log, ends, phys, tot, lp_keep


def draws(ends, n_phy):
    """EndReceive outcomes: m_random.GetValue () > per, with phy j's k-th draw a fixed value."""
    k = np.zeros(n_phy, np.int64)
    ok = np.zeros(n_phy, np.int64)
    for e in ends:
        if e["flags"] & wifi.END_CANCELLED:
            continue
        j = int(e["phy"])
        u = ((k[j] + 1) * 0.6180339887498949 + j * 0.1) % 1.0
        k[j] += 1
        ok[j] += u > e["per"]
    return ok
