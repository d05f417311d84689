"""Extracts tests/golden/general0_v2_node.json from the reference's own recorded
run, simulations/example/results/General-0.{sca,vec} (OMNeT++ 4.6, 2018-06-26;
the only reference-held result files).  Runs in the build container only (the
reference tree is not on the GPU box); the JSON it writes is the fixture.

What the recording pins (a weak, older-code pin: the user side of that run is
mqttApp v1; the fog node is ComputeBrokerApp2, whose 10-ms
timer shows in the data):
  * General-0.sca:273,582,891,1200,1509: ComputeBroker1 received 5 packets, 2..5
    one each (CONNACK only): every forwarded task went to node 0.
  * General-0.vec vector 692 (ComputeBroker1.udp rcvdPk): the CONNACK at
    0.00004688 s and the 4 forwarded tasks' arrival ticks at the node.
  * vector 691 (ComputeBroker1.udp sentPk): the node's 342 sends: CONNECT at 0,
    an advert every 10 ms from CONNACK + 10 ms (ComputeBrokerApp2.cc:219 and
    :261-265), a TaskAck at each task's arrival (:283-288), the timer re-armed
    to arrival + requiredTime (:290-293), then at each firing one release
    (status 6, :222-237) plus an advert: the two-send ticks are the releases.
"""
import json
import os

REF = "/root/reference/simulations/example/results"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "general0_v2_node.json")


def ticks(s: str) -> int:
    """exact decimal seconds -> simtime_t ticks (scale 1e-12)"""
    whole, _, frac = s.partition(".")
    return int(whole) * 10**12 + int((frac + "0" * 12)[:12])


def vector(vid: int):
    rows = []
    with open(os.path.join(REF, "General-0.vec")) as f:
        for ln in f:
            p = ln.rstrip("\n").split("\t")
            if p[0] == str(vid) and len(p) == 4:
                rows.append((ticks(p[2]), int(p[3])))
    return rows


def sca_received():
    got = {}
    with open(os.path.join(REF, "General-0.sca")) as f:
        for no, ln in enumerate(f, 1):
            for k in range(1, 6):
                if ln.startswith(f"scalar WirelessNet.ComputeBroker{k}.udpApp[0] \t\"packets received\""):
                    got[k] = (int(ln.split("\t")[-1]), no)
    return got


def main():
    rcvd = vector(692)
    sent = vector(691)
    recv_sca = sca_received()
    connack, tasks = rcvd[0][0], [t for t, _ in rcvd[1:]]
    send_ticks = [t for t, _ in sent]
    doubles = sorted({t for t in send_ticks if send_ticks.count(t) == 2})
    out = dict(
        source="simulations/example/results/General-0.sca:273,582,891,1200,1509 and General-0.vec vectors 691/692 "
               "(tests/golden/make_general0_fixture.py)",
        packets_received={f"ComputeBroker{k}": v for k, (v, _) in recv_sca.items()},
        packets_received_lines={f"ComputeBroker{k}": no for k, (_, no) in recv_sca.items()},
        connack_tick=connack, task_arrival_ticks=tasks, node_send_ticks=send_ticks, release_ticks=doubles,
        ini=dict(node_mips=1000, broker_mips=1000, send_interval_ms=50, nodes=5,
                 cite="simulations/example/wirelessNet.ini:48,58,62,64"),
        required_time_s=0.01, required_time_cite="mqttApp.cc / mqttApp2.cc:372 (requiredTime = 0.01)",
    )
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")
    print(f"wrote {OUT}: {len(tasks)} tasks, {len(send_ticks)} sends, releases {doubles}")


if __name__ == "__main__":
    main()
