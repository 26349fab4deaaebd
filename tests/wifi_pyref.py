"""A second, independent restatement of the Wi-Fi PHY receive subset in pure Python (test infrastructure).

Small scenarios only.  It cross-checks the C oracle (oracle/nsref_wifi.cc): two restatements written
apart must agree event for event.  Event order: a heap of (ts, uid) keys (scheduler.h:105-121).
Reference lines as in oracle/nsref_wifi.cc: YansWifiPhy::SendPacket (yans-wifi-phy.cc:499-522),
YansWifiChannel::Send (yans-wifi-channel.cc:77-115), StartReceivePacket (yans-wifi-phy.cc:399-496),
InterferenceHelper (interference-helper.cc:171-212, 365-383), WifiPhyStateHelper
(wifi-phy-state-helper.cc:122-183, 254-322, 391-423), EndReceive (yans-wifi-phy.cc:770-799).
"""
import bisect
import heapq
import math

import nsref


def run(sc, durations):
    """sc: wifi.Scenario; durations: ns per transmission.  Returns (stats dict, rx log dict
    {(k, j): (ts, uid, outcome, flags, cca)}, ends list of dicts, tx_base list, phys list of dicts)."""
    n = sc.n_phy
    ed_w = math.pow(10.0, sc.ed / 10.0) / 1000.0
    cca_w = math.pow(10.0, sc.cca / 10.0) / 1000.0
    chain = nsref.loss_chain(*sc.loss)
    phy = [dict(ni_t=[], ni_d=[], first=0.0, rxing=False, end_tx=0, end_rx=0, end_cca=0, live=None,
                rx=0, sync=0, drop_rx=0, drop_tx=0, drop_ed=0, cca_switches=0, end=0, end_cancelled=0, ni_max=0)
           for _ in range(n)]
    heap = []
    for k, t in enumerate(sc.tx):
        heapq.heappush(heap, (int(t["ts"]), int(t["uid"]), ("tx", k)))
    if sc.stop_ts != (1 << 64) - 1:
        heapq.heappush(heap, (sc.stop_ts, sc.stop_uid, ("stop",)))
    uid = sc.uid_start
    st = dict(dispatched=0, tx=0, rx=0, sync=0, drop_rx=0, drop_tx=0, drop_ed=0, cca_evals=0, cca_switches=0,
              end=0, end_cancelled=0, final_ts=0)
    log, ends, tx_base = {}, [], [0] * len(sc.tx)

    def state(p, now):
        if p["end_tx"] > now:
            return "tx"
        if p["rxing"]:
            return "rx"
        if p["end_cca"] > now:
            return "cca"
        return "idle"

    def until_idle(p, now, s):
        r = {"rx": p["end_rx"] - now, "tx": p["end_tx"] - now, "cca": p["end_cca"] - now}.get(s, 0)
        return max(r, 0)

    def ins(p, t, d):  # insert at upper_bound (t)
        i = bisect.bisect_right(p["ni_t"], t)
        p["ni_t"].insert(i, t)
        p["ni_d"].insert(i, d)

    while heap:
        now, euid, ev = heapq.heappop(heap)
        st["dispatched"] += 1
        st["final_ts"] = now
        if ev[0] == "stop":
            break
        if ev[0] == "tx":
            k = ev[1]
            t = sc.tx[k]
            s = int(t["phy"])
            p = phy[s]
            cur = state(p, now)
            assert cur != "tx", "SendPacket while in TX"
            if cur == "rx":
                ends[p["live"]]["flags"] |= 1
                p["rxing"] = False
                p["end_rx"] = now
                p["live"] = None
            p["end_tx"] = now + durations[k]
            st["tx"] += 1
            tx_base[k] = uid
            for j in range(n):
                if j == s or sc.channel[j] != sc.channel[s]:
                    continue
                d = nsref.lib().nsref_distance(*(float(v) for v in (sc.x[s], sc.y[s], sc.z[s], sc.x[j], sc.y[j], sc.z[j])))
                delay = nsref.lib().nsref_const_speed_delay(d, sc.speed)
                rx = nsref.lib().nsref_calc_rx_power(float(t["dbm"]), d, chain)
                heapq.heappush(heap, (now + delay, uid, ("rx", k, j, rx)))
                log[(k, j)] = [now + delay, uid, 255, 0, 0]
                uid += 1
        elif ev[0] == "rx":
            _, k, j, rx = ev
            p = phy[j]
            w = math.pow(10.0, (rx + sc.rx_gain_db) / 10.0) / 1000.0
            end_new = now + durations[k]
            if not p["rxing"]:
                i = bisect.bisect_right(p["ni_t"], now)
                for q in range(i):
                    p["first"] += p["ni_d"][q]
                del p["ni_t"][:i], p["ni_d"][:i]
                p["ni_t"].insert(0, now)
                p["ni_d"].insert(0, w)
            else:
                ins(p, now, w)
            ins(p, end_new, -w)
            p["ni_max"] = max(p["ni_max"], len(p["ni_t"]))
            cur = state(p, now)
            flags, cca, maybe = 0, 0, False
            if cur in ("rx", "tx"):
                outcome = 1 if cur == "rx" else 2
                maybe = end_new > now + until_idle(p, now, cur)
            elif w > ed_w:
                outcome = 0
                p["rxing"] = True
                p["end_rx"] = end_new
                p["live"] = len(ends)
                ends.append(dict(ts=end_new, sync_ts=now, uid=uid, phy=j, tx=k, flags=0))
                heapq.heappush(heap, (end_new, uid, ("end", len(ends) - 1)))
                uid += 1
            else:
                outcome, maybe = 3, True
            if maybe:
                flags |= 1
                noise, end = p["first"], now
                for t_, d_ in zip(p["ni_t"], p["ni_d"]):
                    noise += d_
                    end = t_
                    if end < now:
                        continue
                    if noise < cca_w:
                        break
                cca = end - now if end > now else 0
                if cca:
                    flags |= 2
                    p["end_cca"] = max(p["end_cca"], now + cca)
                    p["cca_switches"] += 1
                    st["cca_switches"] += 1
                st["cca_evals"] += 1
            name = ("sync", "drop_rx", "drop_tx", "drop_ed")[outcome]
            p["rx"] += 1
            p[name] += 1
            st["rx"] += 1
            st[name] += 1
            log[(k, j)][2:] = [outcome, flags, cca]
        else:
            e = ends[ev[1]]
            e["flags"] |= 2
            p = phy[e["phy"]]
            p["end"] += 1
            st["end"] += 1
            if e["flags"] & 1:
                p["end_cancelled"] += 1
                st["end_cancelled"] += 1
            else:
                p["rxing"] = False
                p["live"] = None
    st["next_uid"] = uid
    return st, log, ends, tx_base, phy
