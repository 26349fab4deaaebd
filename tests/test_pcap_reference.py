"""trace.py's pcap writer / reader / diff pinned against the reference's own pcap fixtures:
src/network/test/known.pcap (tests/golden/known.pcap) and pcap-file-test-suite.cc's known packets
(tests/golden/pcap_known_kat.json): ReadFileTestCase (:944-1049) and DiffTestCase (:1053-1101)."""
import json
import os
import struct

import trace

HERE = os.path.dirname(os.path.abspath(__file__))
KNOWN = open(os.path.join(HERE, "golden", "known.pcap"), "rb").read()
KAT = json.load(open(os.path.join(HERE, "golden", "pcap_known_kat.json")))


def test_read_known_pcap():
    hdr, recs = trace.pcap_read(KNOWN)
    assert hdr == (2, 4, 0, 0, 65535, trace.DLT_EN10MB)
    assert len(recs) == len(KAT["packets"])
    for (sec, usec, incl, orig, data), (ks, ku, ki, ko, words) in zip(recs, KAT["packets"]):
        assert (sec, usec, incl, orig) == (ks, ku, ki, ko)
        assert len(data) == incl
        # tcpdump -x prints from the network layer: the words follow the 14-byte Ethernet header
        assert data[14:46] == struct.pack(">16H", *words)


def test_writer_reproduces_known_pcap_bytes():
    """PcapFile::Init + Write (pcap-file.cc:300-381) rebuild the reference's file byte for byte."""
    hdr, recs = trace.pcap_read(KNOWN)
    out = trace.pcap_file_header(snaplen=hdr[4], linktype=hdr[5])
    for sec, usec, _incl, orig, data in recs:
        out += trace.pcap_record(sec, usec, data, total_len=orig, snaplen=hdr[4])
    assert out == KNOWN


def test_diff_known_answers():
    n = KAT["n_packet_bytes"]
    d = trace.pcap_diff(KNOWN, KNOWN)
    assert d[0] is KAT["diff_expected"]["file_vs_itself"]
    # DiffTestCase: f.Init (1, N_PACKET_BYTES), Write (tsSec, tsUsec, data, origLen) of every known packet,
    # where data is the uint16_t[16] array in host (little-endian) byte order
    diff = trace.pcap_file_header(snaplen=n, linktype=1)
    for ts, tu, _i, orig, words in KAT["packets"]:
        diff += trace.pcap_record(ts, tu, struct.pack("<16H", *words), total_len=orig, snaplen=n)
    hdr, recs = trace.pcap_read(diff)
    assert hdr[4] == n and all(r[2] == n for r in recs)
    d = trace.pcap_diff(KNOWN, diff)
    e = KAT["diff_expected"]
    assert d == (e["file_vs_different"], e["sec"], e["usec"])
