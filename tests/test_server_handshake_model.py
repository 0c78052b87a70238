"""The render server's close handshake and stop word as a model (CPU), checked over every interleaving.

The code: hg_mega.hip sv_close / sv_view / sv_wait (device) and hg_runtime.hip server_post_frame / server_stop (host),
DESIGN.md section 4.7b.  Both sides store, then load, with sequentially consistent system-scope atomics, so the model
interleaves whole steps in program order:
  host, posting frame k:  H1 post word := k + 1;  H2 read the closing word;  if raised: H3 read the close word and take
                          the post iff its count >= k + 1
  closing wave:           D1 closing word := 1;  D2 read the post word p;  D3 close word := p | STOP, and every mirror
                          := max(mirror, p | STOP)
The invariant: a post the host takes is one the server traces (its drain count includes it), and a post the server
traces beyond what the host took is never blended (the host re-posts it to a new lifetime).  The stop word's count
(the frames the host asked for) abandons frames posted ahead: a wave's view drops to it once the stop flag is seen."""
import itertools

STOP = 1 << 32


def interleavings(a, b):
    """Every merge of sequences a and b that keeps each one's order."""
    n = len(a) + len(b)
    for pos in itertools.combinations(range(n), len(a)):
        out, ia, ib = [], 0, 0
        for i in range(n):
            if i in pos:
                out.append(a[ia]); ia += 1
            else:
                out.append(b[ib]); ib += 1
        yield out


def run(order, k):
    """One post of frame k (k frames posted before) racing one closing wave."""
    mem = {"post": k, "closing": 0, "closed": None}
    host = {}
    dev = {}
    for step in order:
        if step == "H1":
            mem["post"] = k + 1
        elif step == "H2":
            host["saw_closing"] = mem["closing"]
        elif step == "D1":
            mem["closing"] = 1
        elif step == "D2":
            dev["p"] = mem["post"]
        elif step == "D3":
            mem["closed"] = dev["p"] | STOP
    if host["saw_closing"]:
        taken = (mem["closed"] & 0xFFFFFFFF) >= k + 1  # H3, after D3 (the host waits for the close word)
    else:
        taken = True
    drained = mem["closed"] & 0xFFFFFFFF  # the frames the server traces before its waves leave
    return taken, drained


def test_every_interleaving_keeps_the_invariant():
    for k in (0, 5, 1000):
        seen = set()
        for order in interleavings(["H1", "H2"], ["D1", "D2", "D3"]):
            taken, drained = run(order, k)
            seen.add(taken)
            if taken:  # a taken post is traced
                assert drained >= k + 1, order
            else:  # a refused post was not read by the closer: it is re-posted to a new lifetime, traced there
                assert drained == k, order
        assert seen == {True, False}  # both outcomes occur: the refusal path is real


def test_no_close_means_the_post_is_taken_and_a_later_closer_sees_it():
    for k in (0, 7):
        order = ["H1", "H2", "D1", "D2", "D3"]
        taken, drained = run(order, k)
        assert taken and drained == k + 1


def view_after(mirror_writes, view0):
    """A wave's view (hg_mega.hip sv_view): raised by larger mirror counts; once the stop flag is in the mirror, set
    to the stop word's count (which may be lower: frames posted ahead are abandoned)."""
    mirror, view = 0, view0
    for w in mirror_writes:
        mirror = max(mirror, w)
        count = mirror & 0xFFFFFFFF
        if count > view or (mirror & STOP and count != view):
            view = count
    return view, bool(mirror & STOP)


def test_stop_word_abandons_frames_posted_ahead_and_keeps_committed_ones():
    committed, posted = 10, 14  # 4 frames traced ahead of the host's calls
    # the pollers raised the mirror to the posted count; then the host's stop word carries the committed count
    for order in itertools.permutations([posted, committed | STOP]):
        view, stop = view_after(list(order), view0=0)
        assert stop and view == committed
    # a closing wave published the posted count with the stop flag: the waves drain every posted frame (harmless:
    # only committed frames are blended), and a later host stop word cannot lower it below what was already published
    view, stop = view_after([posted, posted | STOP, committed | STOP], view0=posted)
    assert stop and view == posted
    # never below a committed frame: every stop word carries at least the committed count
    for extra in range(0, 5):
        view, _ = view_after([committed + extra, committed | STOP], view0=committed + extra)
        assert view >= committed
