// macstub.cc — measurement tool (not part of the product): the closed-loop Wi-Fi bench's MAC stand-in as C
// callbacks on the host-closure runtime (lib/libnsgpu_macstub.so, bench.py --workload wifi-loop).
//
// The same stand-in tests/wifi_loop_harness.py runs in Python and the oracle's nsref_wifil_mac in C++: per phy
// an attempt reads the PHY state (WifiPhyStateHelper::GetState through nsgpu_sim_wifi_state), sends one frame
// when the PHY is IDLE and tries again a period later, else counts a busy attempt and tries again after the
// phy's backoff.  The first attempts are scheduled in phy order at setup.  In ns-3 the MAC (DcfManager,
// dcf-manager.cc:591-641) is C++ as well: a Python closure per host event is this harness's overhead, not the
// engine's, so the bench line says which stand-in ran.
#include <cstdint>
#include <vector>

#include "nsgpu.h"

namespace {
struct Stub {
  nsgpu_sim *sim;
  std::vector<uint64_t> backoff;
  uint64_t period;
  uint32_t size, modclass, bw, preamble;
  uint64_t rate;
  double dbm;
  uint64_t sends = 0, busy = 0;
  int err = 0;  // the first failing call's status (the run goes on; the caller reads it)
};

void attempt(void *user, uint64_t phy) {
  Stub *m = static_cast<Stub *>(user);
  const uint32_t i = (uint32_t)phy;
  nsgpu_wifil_phy_state st;
  int rc = nsgpu_sim_wifi_state(m->sim, i, &st);
  if (rc == 0 && st.state != NSGPU_WIFIL_IDLE) {
    m->busy++;
    rc = nsgpu_sim_schedule(m->sim, (int64_t)m->backoff[i], attempt, m, phy, nullptr);
  } else if (rc == 0) {
    rc = nsgpu_sim_wifi_send(m->sim, i, m->size, m->dbm, m->modclass, m->rate, m->bw, m->preamble);
    if (rc == 0) m->sends++;
    if (rc == 0) rc = nsgpu_sim_schedule(m->sim, (int64_t)m->period, attempt, m, phy, nullptr);
  }
  if (rc && !m->err) m->err = rc;
}
}  // namespace

extern "C" {
// Schedules every phy's first attempt (phy order) on `sim`, whose Wi-Fi PHYs are attached.
int nsgpu_macstub_install(nsgpu_sim *sim, uint32_t n_phy, const uint64_t *first, const uint64_t *backoff,
                          uint64_t period, uint32_t size, double dbm, uint32_t modclass, uint64_t rate, uint32_t bw,
                          uint32_t preamble, void **out) {
  if (!sim || !first || !backoff || !out) return NSGPU_EINVAL;
  Stub *m = new Stub{sim, std::vector<uint64_t>(backoff, backoff + n_phy), period, size, modclass, bw, preamble, rate, dbm};
  for (uint32_t i = 0; i < n_phy; i++) {
    const int rc = nsgpu_sim_schedule(sim, (int64_t)first[i], attempt, m, i, nullptr);
    if (rc) {
      delete m;
      return rc;
    }
  }
  *out = m;
  return NSGPU_OK;
}
// Sends, busy attempts, and the first failing runtime call's status (0: none).
int nsgpu_macstub_counts(void *h, uint64_t *sends, uint64_t *busy, int *err) {
  const Stub *m = static_cast<const Stub *>(h);
  if (!m || !sends || !busy || !err) return NSGPU_EINVAL;
  *sends = m->sends;
  *busy = m->busy;
  *err = m->err;
  return NSGPU_OK;
}
int nsgpu_macstub_destroy(void *h) {
  delete static_cast<Stub *>(h);
  return NSGPU_OK;
}
}
