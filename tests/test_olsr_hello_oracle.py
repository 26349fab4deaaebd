"""The reference's point-to-point HELLO pcaps (src/olsr/test/olsr-hello-regression-test-{0,1}-1.pcap) rebuilt by
the oracle's device chain from the replayed sends (tests/olsr_hello_replay.py): every record's microsecond, length
and order, then the files byte for byte.  No GPU."""
import olsr_hello_replay as hello


def test_oracle_rebuilds_the_hello_pcaps():
    files, recs, sends = hello.golden()
    assert len(sends) == 6 and {L for _t, _i, L, _r in sends} == {50, 58}
    sc, st, _devc, appc, _log, tr = hello.oracle_run()
    assert int(appc["rx_packets"][:2].sum()) == 6  # (the PacketSinks on port 698)
    out = hello.rebuild(files, recs, hello.sniffer_records(sc, tr))
    assert out[0] == files[0] and out[1] == files[1]


def test_sub_microsecond_offsets_follow_int64x64():
    """A 50-byte frame's transmission time is Seconds (8e-5), which int64x64 makes 79,999 ns (nstime.h:586-589),
    so its reception lands in the recorded microsecond only when the send is >= 1 ns into its own."""
    import nsref
    assert nsref.seconds(50 * 8 / hello.BPS) == 79_999
    _files, _recs, sends = hello.golden()
    ts = hello.schedule(sends)
    assert all(t % 1000 in (1, 201) or t % 1000 == 0 for t in ts)
