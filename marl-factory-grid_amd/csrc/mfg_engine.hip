// mfg_engine.hip — MI355X (gfx950) batched step engine for the marl-factory-grid world: host side (C-ABI of
// include/mfg.h, launch shapes, spec upload). Device code: mfg_kernels.h; the observation-render instantiations:
// mfg_obs_*.hip.
#include "mfg_kernels.h"

// ================================================================================================
// host side: C-ABI (include/mfg.h)
// ================================================================================================
static int wpb_for(size_t lds);  // waves per workgroup for a per-wave LDS slice (launch shape, below)

struct mfg_engine {
  int device = 0;
  long long B = 0;
  MfgDevSpec h{};
  MfgDevSpec* d_spec = nullptr;
  std::vector<void*> d_bufs;
  uint8_t* d_state = nullptr;
  int maxpts = 0;
  // per-kernel timing (mfg_profile)
  bool prof = false;
  std::vector<hipEvent_t> ev_free;
  int rd_slot = 0;     // done list k_logic appends to (alternates per step)
  int rd_blocks = 1;   // k_resetdone workgroups (occupancy x CUs)
  int rpd_blocks = 1;  // k_replay_done workgroups (one wave each)
  int* rp_hist = nullptr;  // replay order by debt : RP_NB bucket counts / offsets
  int* rp_order = nullptr;  // [B] envs in launch order
  uint8_t* rp_key = nullptr;  // [B] bucket per env
  hipStream_t aux = nullptr;  // second stream: resets of a step's done envs and their render (MFG_RESET_OVERLAP)
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  int obs_list_blocks = 1;  // workgroups of the done-list render (resident grid, strides over the list)
  int n_cu = 1;
  bool overlap = false;     // resets beside the render (MFG_RESET_OVERLAP)
  bool replay_each = false; // pay the shuffle debt after every step, not once per call (long resets + in-step RNG)
  int obs_nwv = 1;          // waves per env of the render (> 1: multi-wave render, k_obs_mw)
  bool replay2 = false;     // two-wave replay (k_replay2) for floor lists whose 1-wave slice fills a SIMD
  struct Mark { int k; hipEvent_t a, b; };
  std::vector<Mark> marks;
  std::string err;  // mfg_last_error(e)
};

static hipEvent_t prof_event(mfg_engine* e) {
  if (!e->ev_free.empty()) {
    hipEvent_t ev = e->ev_free.back();
    e->ev_free.pop_back();
    return ev;
  }
  hipEvent_t ev = nullptr;
  if (hipEventCreate(&ev) != hipSuccess) return nullptr;
  return ev;
}
// bracket one launch with events when profiling (PROF_BEGIN before, PROF_END after the launch)
#define PROF_BEGIN(E, ST) hipEvent_t _pa = nullptr; if ((E)->prof) { _pa = prof_event(E); if (_pa) (void)hipEventRecord(_pa, ST); }
#define PROF_END(E, ST, KID) if (_pa) { hipEvent_t _pb = prof_event(E); if (_pb) { (void)hipEventRecord(_pb, ST); (E)->marks.push_back({KID, _pa, _pb}); } }

static thread_local std::string g_err;
static int fail(const std::string& m) {
  g_err = m;
  return -1;
}
#define HIPCHK(x)                                                               \
  do {                                                                          \
    hipError_t _e = (x);                                                        \
    if (_e != hipSuccess) return fail(std::string(#x) + ": " + hipGetErrorString(_e)); \
  } while (0)

extern "C" const char* mfg_last_error(const mfg_engine* e) { return e ? e->err.c_str() : g_err.c_str(); }

// Entry points run on the engine's device and give the caller's current device back (mfg.h, mfg_create).
struct DevGuard {
  int prev = -1;
  explicit DevGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DevGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};
// run an engine entry point on its device; a failure's message is kept per engine
#define ENGINE_CALL(E, CALL)                 \
  do {                                       \
    if (!(E)) return fail("null engine");    \
    DevGuard _g((E)->device);                \
    const int _rc = (CALL);                  \
    if (_rc) (E)->err = g_err;               \
    return _rc;                              \
  } while (0)

extern "C" int mfg_decode_events(const uint8_t* ev_act, const uint8_t* ev_watch, const int32_t* ev_misc, int n_agents,
                                 mfg_events* out) {
  if (!ev_act || !ev_watch || !ev_misc || !out) return fail("null argument");
  if (n_agents < 1 || n_agents > MFG_MAX_AGENTS) return fail("n_agents out of range");
  memset(out, 0, sizeof(*out));
  for (int a = 0; a < n_agents; a++) { out->act[a] = ev_act[a]; out->watch[a] = ev_watch[a]; }
  const int32_t* m = ev_misc;
  out->door_coll = (uint64_t)(uint32_t)m[MFG_EVM_DOOR_COLL_LO] | ((uint64_t)(uint32_t)m[MFG_EVM_DOOR_COLL_HI] << 32);
  out->door_coll_hi = (uint64_t)(uint32_t)m[MFG_EVM_DOOR_COLL_2] | ((uint64_t)(uint32_t)m[MFG_EVM_DOOR_COLL_3] << 32);
  out->maint_coll = (uint64_t)(uint32_t)m[MFG_EVM_MAINT_COLL] | ((uint64_t)(uint32_t)m[MFG_EVM_MAINT_COLL_HI] << 32);
  out->respawn_items_value = m[MFG_EVM_RESPAWN_ITEMS];
  out->dirt_spawn_value = m[MFG_EVM_DIRT_SPAWN];
  out->dirt_spawn_valid = m[MFG_EVM_DIRT_VALID];
  out->dest_reached = m[MFG_EVM_DEST_REACHED];
  out->door_autoclose = m[MFG_EVM_FLAGS] & 1;
  out->crashed = (m[MFG_EVM_FLAGS] >> 1) & 1;
  out->crash_reason = (m[MFG_EVM_FLAGS] >> 8) & 0xFF;
  out->done_mask = m[MFG_EVM_DONE_MASK];
  out->step = m[MFG_EVM_STEP];
  out->episode = m[MFG_EVM_EPISODE];
  out->maint_base = m[MFG_EVM_MAINT_BASE];
  return 0;
}

template <typename T>
static int upload(mfg_engine* e, const T* src, size_t n, const T** dst) {
  void* p = nullptr;
  HIPCHK(hipMalloc(&p, sizeof(T) * (n ? n : 1)));
  if (n) HIPCHK(hipMemcpy(p, src, sizeof(T) * n, hipMemcpyHostToDevice));
  e->d_bufs.push_back(p);
  *dst = (const T*)p;
  return 0;
}

// numpy SeedSequence(entropy) -> PCG64 initial state (numpy/random/bit_generator.pyx, pcg64.h)
static void pcg64_seed(uint32_t entropy, uint64_t* st_hi, uint64_t* st_lo, uint64_t* inc_hi, uint64_t* inc_lo) {
  auto hashmix = [](uint32_t v, uint32_t& hc) {
    v ^= hc; hc *= 0x931e8875u; v *= hc; v ^= v >> 16; return v;
  };
  auto mix = [](uint32_t x, uint32_t y) {
    uint32_t r = 0xca01f9ddu * x - 0x4973f715u * y; r ^= r >> 16; return r;
  };
  uint32_t pool[4], hc = 0x43b0d7e5u;
  pool[0] = hashmix(entropy, hc);
  for (int i = 1; i < 4; i++) pool[i] = hashmix(0u, hc);
  for (int s = 0; s < 4; s++)
    for (int d = 0; d < 4; d++)
      if (s != d) pool[d] = mix(pool[d], hashmix(pool[s], hc));
  uint32_t st[8], hb = 0x8b51f9ddu;
  for (int i = 0; i < 8; i++) {
    uint32_t v = pool[i % 4];
    v ^= hb; hb *= 0x58f38dedu; v *= hb; v ^= v >> 16;
    st[i] = v;
  }
  uint64_t w[4];
  for (int i = 0; i < 4; i++) w[i] = (uint64_t)st[2 * i] | ((uint64_t)st[2 * i + 1] << 32);
  typedef unsigned __int128 u128;
  const u128 mult = ((u128)2549297995355413924ULL << 64) | 4865540595714422341ULL;
  u128 seed = ((u128)w[0] << 64) | w[1], inc = ((((u128)w[2] << 64) | w[3]) << 1) | 1u;
  u128 state = 0;
  state = state * mult + inc;
  state += seed;
  state = state * mult + inc;
  *st_hi = (uint64_t)(state >> 64); *st_lo = (uint64_t)state;
  *inc_hi = (uint64_t)(inc >> 64); *inc_lo = (uint64_t)inc;
}

static int align_up(int x, int a) { return (x + a - 1) / a * a; }

static void make_layout(const mfg_spec* s, MfgLayout* L, int imax, int pmax, int dropmax, int destmax, int mmax,
                        int kmax, int mstate_ints, int path_cap, int graph, int dirt_cap) {
  // [0, o_logic): what a step reads and writes (k_logic stages only this prefix); [o_logic, o_mt): the
  // per-episode values only the render reads (frozen ray origins, positions, batteries, Q11/Q12); then the RNG
  // streams and the maintainer tail. Rule counters: one per rule of the spec.
  int o = 0;
  const int A = s->n_agents, nd = s->n_doors;
  const int dm = dirt_cap;
  L->o_hdr = o; o += 4 * MFG_HDR_N;
  L->o_rule_ctr = o; o += 4 * std::max(1, s->n_rules);
  L->o_agent_pos = o; o += 4 * A;
  L->o_agent_arr = o; o += 4 * A;
  L->o_agent_par = o; o += 4 * A;
  L->o_door = o; o += 4 * nd;
  L->o_items = o; o += 4 * imax;
  L->o_pods = o; o += 4 * pmax;
  L->o_drops = o; o += 4 * dropmax;
  L->o_dests = o; o += 4 * destmax;
  L->o_machines = o; o += 4 * mmax;
  L->o_maints = o; o += 4 * kmax;
  L->o_dirt_pos = o; o += 4 * dm;
  L->o_dirt_id = o; o += 4 * dm;
  o = align_up(o, 8);
  L->o_battery = o; o += 8 * A;
  L->o_dirt_amt = o; o += 8 * dm;
  L->o_pcg = o; o += 8 * 4;
  o = align_up(o, 16);
  L->o_logic = o;
  L->o_frozen_org = o; o += 4 * A;
  L->o_frozen_gp = o; o += 4 * A;
  o = align_up(o, 8);
  L->o_frozen_bat = o; o += 8 * A;
  o = align_up(o, 16);
  L->o_mt = o; o += 4 * 624;
  L->o_perm = o; o += std::max(2 * s->n_floor, 128);  // >= 128 B after MT: mt_twist reads up to word 652 (dropped)
  o = align_up(o, 4);
  L->o_mstate = o; o += 4 * kmax * mstate_ints;
  L->o_mpath = o; o += 2 * kmax * path_cap;
  o = align_up(o, 4);
  L->o_grank = o; o += graph ? 2 * s->n_floor : 0;
  L->size = align_up(o, 16);
}

// Probe: does one ds_wrxchg with conflicting addresses apply its lanes in ascending lane order (each
// lane gets the previous same-address lane's value back, the last lane's value stays)? The exchange
// path of the shuffle blocks relies on it; without it the table path is used.
__global__ void __launch_bounds__(64) k_probe_xchg(int* bad) {
  __shared__ uint32_t tab[64];
  const int lane = lane_id();
  int nbad = 0;
  for (int it = 1; it <= 64; it++) {
    tab[lane] = 1000u + lane;
    wave_sync();
    const int a = (int)((lane * 2654435761u + it * 40503u) >> 7) % it;  // many conflicts, varied patterns
    const uint32_t old = atomicExch(&tab[a], (uint32_t)lane);
    wave_sync();
    // expected: the previous lane with the same address, or the initial value
    int prev = -1;
    for (int l = 0; l < lane; l++)
      if ((int)((l * 2654435761u + it * 40503u) >> 7) % it == a) prev = l;
    const uint32_t want = prev >= 0 ? (uint32_t)prev : 1000u + a;
    int last = -1;
    for (int l = 0; l < 64; l++)
      if ((int)((l * 2654435761u + it * 40503u) >> 7) % it == lane) last = l;
    const uint32_t want_fin = last >= 0 ? (uint32_t)last : 1000u + lane;
    nbad += (old != want) + (tab[lane] != want_fin);
    wave_sync();
  }
  // the same for 16-bit exchanges through ds_mskor_rtn_b32 (two entries per word, both halves conflict)
  __shared__ uint16_t tab16[64];
  for (int it = 1; it <= 64; it++) {
    tab16[lane] = (uint16_t)(1000 + lane);
    wave_sync();
    const int a = (int)((lane * 2246822519u + it * 3266489917u) >> 9) % it;
    const uint32_t old = lds_xchg_u16(&tab16[a], (uint32_t)lane);
    wave_sync();
    int prev = -1;
    for (int l = 0; l < lane; l++)
      if ((int)((l * 2246822519u + it * 3266489917u) >> 9) % it == a) prev = l;
    const uint32_t want = prev >= 0 ? (uint32_t)prev : 1000u + a;
    int last = -1;
    for (int l = 0; l < 64; l++)
      if ((int)((l * 2246822519u + it * 3266489917u) >> 9) % it == lane) last = l;
    const uint32_t want_fin = last >= 0 ? (uint32_t)last : 1000u + lane;
    nbad += (old != want) + ((uint32_t)tab16[lane] != want_fin);
    wave_sync();
  }
  atomicAdd(bad, nbad);
}

static int probe_xchg_order(int device) {
  (void)device;
  int* d = nullptr;
  int h = -1;
  if (hipMalloc((void**)&d, sizeof(int)) != hipSuccess) return 0;
  if (hipMemset(d, 0, sizeof(int)) == hipSuccess) {
    hipLaunchKernelGGL(k_probe_xchg, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(&h, d, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) h = -1;
  }
  (void)hipFree(d);
  return h == 0 ? 1 : 0;
}

// every bounded count of a caller-built spec (the kernels index fixed-size spec arrays with them)
static int validate_spec(const mfg_spec* s) {
  if (s->abi_version != MFG_ABI_VERSION) return fail("spec ABI version mismatch");
  if (s->H < 1 || s->W < 1 || !s->level) return fail("empty level");
  if (s->H * s->W > 65535) return fail("level too large for 16-bit cell indices");
  if (s->n_agents < 1 || s->n_agents > MFG_MAX_AGENTS) return fail("n_agents out of range");
  if (s->n_doors < 0 || s->n_doors > MFG_MAX_DOORS) return fail("too many doors");
  if (s->n_floor < 1 || s->n_floor > s->H * s->W || !s->floor_cells) return fail("n_floor out of range");
  if (s->n_walls < 0 || s->n_walls > s->H * s->W) return fail("n_walls out of range");
  // the ray radius is the window diameter (Q13): 2 r + 1, or min(H, W) with full observability; a ray holds
  // radius + 1 points: up to 64 the walk keeps them in one 32- or 64-bit mask (k_obs), up to 255 the long-ray render
  // walks 32-point segments (k_obs_lr)
  if (s->pomdp_r < 0 || s->pomdp_r > 126) return fail("engine supports pomdp_r in [0, 126] (rays of <= 255 points)");
  if (s->pomdp_r == 0 && std::min(s->H, s->W) > 254)
    return fail("full observability (pomdp_r 0) needs min(H, W) <= 254 (rays of <= 255 points)");
  for (int a = 0; a < s->n_agents; a++) {
    if (s->n_positions[a] < 0 || s->n_positions[a] > MFG_MAX_POSITIONS) return fail("n_positions out of range");
    for (int k = 0; k < s->n_positions[a]; k++)
      if (s->positions[a][k] < 0 || s->positions[a][k] >= s->H * s->W) return fail("agent position out of range");
  }
  if (s->n_dest_entries < 0 || s->n_dest_entries > MFG_MAX_AGENTS) return fail("n_dest_entries out of range");
  for (int j = 0; j < s->n_dest_entries; j++) {
    if (s->dest_entry_agent[j] < 0 || s->dest_entry_agent[j] >= s->n_agents) return fail("dest entry agent out of range");
    if (s->dest_entry_q[j] < 0 || s->dest_entry_n[j] < 0 || s->dest_entry_n[j] > MFG_MAX_POSITIONS)
      return fail("dest entry count out of range");
    if (!s->dest_entry_q[j] && !s->dest_entry_n[j]) return fail("dest entry without positions");
    for (int k = 0; k < s->dest_entry_n[j]; k++)
      if (s->dest_entry_cells[j][k] < 0 || s->dest_entry_cells[j][k] >= s->H * s->W) return fail("dest cell out of range");
  }
  if (s->n_rays < 1 || !s->ray_off || !s->ray_pts) return fail("empty ray table");
  if (s->n_rules < 0 || s->n_rules > MFG_MAX_RULES) return fail("n_rules out of range");
  for (int a = 0; a < s->n_agents; a++) {
    if (s->n_actions[a] < 1 || s->n_actions[a] > MFG_MAX_ACTIONS) return fail("n_actions out of range");
    if (s->n_layers[a] < 0 || s->n_layers[a] > MFG_MAX_LAYERS) return fail("n_layers out of range");
    if (s->combined_n[a] < 0 || s->combined_n[a] > MFG_MAX_COMBINED) return fail("combined_n out of range");
    for (int j = 0; j < s->n_actions[a]; j++) {
      const mfg_action& ac = s->actions[a][j];
      if (ac.op < MFG_ACT_NOOP || ac.op > MFG_ACT_MACHINE) return fail("unknown action opcode");
      if (ac.op == MFG_ACT_MOVE && (ac.arg < 0 || ac.arg > 7)) return fail("move direction out of range");
    }
    for (int l = 0; l < s->n_layers[a]; l++) {
      const int k = s->layers[a][l].kind, t = s->layers[a][l].tag;
      if (k < MFG_LAYER_ZERO || k > MFG_LAYER_GLOBALPOS) return fail("unknown layer kind");
      if (k == MFG_LAYER_TAG && !((t >= 0 && t <= MFG_TAG_MAINTAINERS) ||
                                  (t >= MFG_TAG_AGENT0 && t < MFG_TAG_AGENT0 + s->n_agents)))
        return fail("layer tag out of range");
    }
    for (int q = 0; q < s->combined_n[a]; q++) {
      const int t = s->combined_tags[a][q];
      if (!((t >= 0 && t <= MFG_TAG_MAINTAINERS) || (t >= MFG_TAG_AGENT0 && t < MFG_TAG_AGENT0 + s->n_agents)))
        return fail("combined tag out of range");
    }
  }
  for (int r = 0; r < s->n_rules; r++)
    if (s->rules[r].op < MFG_RULE_SPAWN_BATTERIES || s->rules[r].op > MFG_RULE_RANDOM_INIT_STEPS)
      return fail("unknown rule opcode");
  for (int f = 0; f < s->n_floor; f++)
    if (s->floor_cells[f] < 0 || s->floor_cells[f] >= s->H * s->W) return fail("floor cell out of range");
  for (int w = 0; w < s->n_walls; w++)
    if (!s->wall_cells || s->wall_cells[w] < 0 || s->wall_cells[w] >= s->H * s->W) return fail("wall cell out of range");
  for (int d = 0; d < s->n_doors; d++)
    if (!s->door_cells || s->door_cells[d] < 0 || s->door_cells[d] >= s->H * s->W) return fail("door cell out of range");
  return 0;
}

static int create_impl(const mfg_spec* s, int device, int64_t n_envs, const mfg_variant& v, mfg_engine** out);
extern "C" int mfg_create_variant(const mfg_spec* s, int device, int64_t n_envs, const mfg_variant* v,
                                  mfg_engine** out) {
  if (!s || !out) return fail("null argument");
  if (n_envs < 1) return fail("n_envs must be >= 1");
  if (validate_spec(s)) return -1;
  const mfg_variant none{0, 0, 0, 0, 0, 0};
  DevGuard g(device);
  return create_impl(s, device, n_envs, v ? *v : none, out);
}
extern "C" int mfg_create(const mfg_spec* s, int device, int64_t n_envs, mfg_engine** out) {
  return mfg_create_variant(s, device, n_envs, nullptr, out);
}

static int create_impl(const mfg_spec* s, int device, int64_t n_envs, const mfg_variant& v, mfg_engine** out) {
  auto* e = new mfg_engine();
  e->device = device;
  e->B = n_envs;
  if (hipSetDevice(device) != hipSuccess) { delete e; return fail("hipSetDevice failed"); }
  MfgDevSpec& h = e->h;
  h.s = *s;
  const int HW = s->H * s->W;
  h.HW = HW; h.nf = s->n_floor; h.nw = s->n_walls; h.nd = s->n_doors; h.A = s->n_agents;
  // window (observation_builder.py:51): (2r+1)^2, or the level with full observability; ray radius min(window)
  h.r = s->pomdp_r;
  h.oh = s->pomdp_r ? 2 * s->pomdp_r + 1 : s->H;
  h.ow = s->pomdp_r ? 2 * s->pomdp_r + 1 : s->W;
  h.dd = h.oh * h.ow;
  h.fr = std::min(h.oh, h.ow);
  h.nrays = s->n_rays;
  h.lane_passes = (s->n_agents > MFG_WAVE || s->n_doors > MFG_WAVE) ? 2 : 1;
  for (int a = 0; a < s->n_agents; a++) {  // combined layers that are plain member counts (MfgDevSpec)
    uint32_t tm = 0;
    uint64_t am[2] = {0, 0};
    bool fast = true;
    for (int q = 0; q < s->combined_n[a]; q++) {
      const int t = s->combined_tags[a][q];
      if (t >= MFG_TAG_AGENT0) {
        const int b = t - MFG_TAG_AGENT0;
        const uint64_t bit = 1ull << (b & 63);
        fast = fast && !(am[b >> 6] & bit);
        am[b >> 6] |= bit;
      } else {
        const bool unit = t != MFG_TAG_DOORS && t != MFG_TAG_DIRT && t != MFG_TAG_MACHINES;
        fast = fast && unit && !(tm & (1u << t));
        tm |= 1u << t;
      }
    }
    h.comb_fast[a] = fast && s->combined_n[a] > 0;
    h.comb_unit_tags[a] = tm;
    h.comb_agents[a] = am[0];
    h.comb_agents2[a] = am[1];
  }
  if (h.nrays > 4 * MFG_WAVE) { delete e; return fail("more than 256 rays"); }
  {  // points per ray (<= fr + 1), rounded up to a compiled k_obs instantiation (DISPATCH_MP)
    int mp = 1;
    for (int r = 0; r < h.nrays; r++) mp = std::max(mp, s->ray_off[r + 1] - s->ray_off[r]);
    if (mp > 255) { delete e; return fail("rays longer than 255 points"); }
    static const int SIZES[] = {4, 6, 8, 10, 12, 14, 16, 18, 24, 32, 48, 64};
    h.maxpts = 0;  // 0: the long-ray render (k_obs_lr, 32-point segments of a 16-bit ray table)
    // more than 64 agents: always the long-ray render, the one render compiled with the second agent word (its
    // per-agent tables live in HBM pool slots, so they do not cost the other renders' occupancy)
    if (s->n_agents <= MFG_WAVE)
      for (int k : SIZES) if (k >= mp) { h.maxpts = k; break; }
    h.lrpts = h.maxpts ? 0 : align_up(mp, 32);
  }
  int lmax = 1;
  for (int a = 0; a < s->n_agents; a++) lmax = s->n_layers[a] > lmax ? s->n_layers[a] : lmax;
  h.lmax = lmax;
  h.obs_agent_stride = lmax * h.dd;
  int imax = 0, pmax = 0, dropmax = 0, destmax = 0, mmax = 0, kmax = 0, moving = 0;
  for (int r = 0; r < s->n_rules; r++) {
    const mfg_rule& ru = s->rules[r];
    if (ru.op == MFG_RULE_SPAWN_ITEMS) imax = ru.i[0];
    if (ru.op == MFG_RULE_SPAWN_PODS) pmax = ru.i[0];
    if (ru.op == MFG_RULE_SPAWN_DROPOFFS) dropmax = ru.i[0];
    if (ru.op == MFG_RULE_SPAWN_DESTS) destmax = ru.i[0];
    if (ru.op == MFG_RULE_SPAWN_DEST_ON_AGENT) destmax = s->n_agents;
    if (ru.op == MFG_RULE_SPAWN_DEST_PER_AGENT) destmax = s->n_dest_entries;
    if (ru.op == MFG_RULE_SPAWN_MACHINES) mmax = ru.i[0];
    if (ru.op == MFG_RULE_SPAWN_MAINTAINERS) kmax = ru.i[0];
    if (ru.op == MFG_RULE_MOVE_MAINTAINERS) moving = 1;
  }
  if (imax > 64 || pmax > 64 || dropmax > 64 || destmax > 64 || mmax > 30 || kmax > 64) {
    delete e; return fail("group quantity too large for the engine");
  }
  h.imax = imax; h.pmax = pmax; h.dropmax = dropmax; h.destmax = destmax; h.mmax = mmax; h.kmax = kmax;
  h.mstate_ints = MS_NEXT + mmax + 1;
  h.path_cap = moving ? std::min(std::min(4 * (s->H + s->W), s->n_floor), 1000) : 0;  // route fits the 2 KB scratch
  // dirt-pile slots: the initial spawn plus every respawn one episode can hold (DoneAtMaxStepsReached bounds
  // it; without it the engine's maximum). More piles than slots flag the env (H_OVERFLOW), never silently.
  int dirt_q = 0;
  h.dirt_cap = 0;
  if (s->has_dirt) {
    int max_steps = -1, respawn_n = 0, freq = 0;
    for (int r = 0; r < s->n_rules; r++) {
      if (s->rules[r].op == MFG_RULE_DONE_MAXSTEPS) max_steps = s->rules[r].i[0];
      if (s->rules[r].op == MFG_RULE_RESPAWN_DIRT) { freq = s->rules[r].i[0]; respawn_n = s->rules[r].i[1]; }
    }
    dirt_q = std::max(s->dirt_quantity, respawn_n);
    long long need = (long long)s->dirt_quantity + 1;
    if (respawn_n > 0) need = max_steps < 0 ? MFG_DIRT_MAX : need + (long long)(max_steps / (freq + 1) + 1) * (respawn_n + 1);
    h.dirt_cap = (int)std::min<long long>(MFG_DIRT_MAX, std::max<long long>(MFG_WAVE, (need + 63) / 64 * 64));
  }
  // per-wave LDS scratch: spawn positions + amounts of the largest dirt spawn, maintainer routes, >= 2 KB
  int dest_list = 0;  // SpawnDestinationsPerAgent candidate list after the shuffle sinks (quantity mode: the floor)
  for (int j = 0; j < s->n_dest_entries; j++) dest_list = std::max(dest_list, s->dest_entry_q[j] ? 2 * s->n_floor : 64);
  h.scratch_bytes = align_up(std::max({2048, 12 * (dirt_q + 2) + 16, 2 * (h.path_cap + 2), 128 + dest_list + 64}), 16);
  make_layout(s, &h.L, imax, pmax, dropmax, destmax, mmax, kmax, h.mstate_ints, h.path_cap, moving, h.dirt_cap);
  // per-phase rule lists (rule_tick_step / rule_post_step / rule_check_done act only for these ops)
  for (int r = 0; r < s->n_rules; r++) {
    const int op = s->rules[r].op;
    const bool tick = op == MFG_RULE_DOOR_AUTOCLOSE || op == MFG_RULE_RESPAWN_ITEMS || op == MFG_RULE_BATTERY_DECHARGE ||
                      op == MFG_RULE_DONE_BATTERY || op == MFG_RULE_RESPAWN_DIRT || op == MFG_RULE_MOVE_MAINTAINERS ||
                      op == MFG_RULE_DEST_REACH || op == MFG_RULE_DONE_DEST;
    const bool post = op == MFG_RULE_RESPAWN_ITEMS || op == MFG_RULE_WATCH_COLLISIONS || op == MFG_RULE_BATTERY_DECHARGE ||
                      op == MFG_RULE_DONE_BATTERY;
    const bool done = op == MFG_RULE_DONE_MAXSTEPS || op == MFG_RULE_WATCH_COLLISIONS || op == MFG_RULE_DONE_BATTERY ||
                      op == MFG_RULE_DONE_MAINT_COLLISION || op == MFG_RULE_DONE_DIRT || op == MFG_RULE_DONE_DEST;
    if (tick) h.ph_rule[0][h.n_ph[0]++] = (uint8_t)r;
    if (post) h.ph_rule[1][h.n_ph[1]++] = (uint8_t)r;
    if (done) h.ph_rule[2][h.n_ph[2]++] = (uint8_t)r;
  }
  h.step_rng = 0;
  for (int r = 0; r < s->n_rules; r++)  // dirt spawns and maintainer retargets consume the floor order mid-step
    if (s->rules[r].op == MFG_RULE_RESPAWN_DIRT || s->rules[r].op == MFG_RULE_MOVE_MAINTAINERS) h.step_rng = 1;
  h.respawn_mask = 0;
  for (int r = 0; r < s->n_rules && r < 32; r++)
    if (s->rules[r].op == MFG_RULE_RESPAWN_DIRT) h.respawn_mask |= 1u << r;
  h.map_bytes = align_up(2 * HW, 16);
  h.map_bytes8 = align_up(HW, 16);
  h.lds_full = align_up(h.L.size + h.scratch_bytes + 4 * MFG_STAB_N, 16);
  // BFS scratch of the maintainer routing: pred, succ, two fringes, level copy (u16 each) + discovery keys;
  // in the LDS slice when it fits, else a per-env HBM pool (grid128: 212 KB per env)
  h.bfs_bytes = moving ? align_up(10 * h.nf + 4 * h.nf + 64, 16) : 0;
  h.bfs_off = 0;
  h.bfs_pool = nullptr;
  // (mfg_variant.bfs_hbm: the HBM pool path on small levels too, for the parity tests)
  const bool bfs_lds = moving && h.lds_full + h.bfs_bytes <= MFG_LDS_MAX && !v.bfs_hbm;
  if (bfs_lds) {
    h.bfs_off = h.lds_full;
    h.lds_full = align_up(h.lds_full + h.bfs_bytes, 16);
  }
  // identifier-collision pairs of the obs dedupe: per int-id entity one wall and one door partner and at
  // most one partner per other kind (identifiers are unique within a kind), plus the static Wall/Door pairs
  {
    const int tot_cap = imax + pmax + dropmax + destmax + h.dirt_cap + mmax + kmax;
    h.max_pairs = std::max(16, 2 * tot_cap + 3 * tot_cap);
  }
  h.pair_pool = nullptr;
  h.lds_logic = h.step_rng ? h.lds_full : h.L.o_logic + 4 * MFG_WAVE * h.lane_passes;  // step prefix + per-door count scratch
  h.fv_words = align_up((2 * h.fr + 1) * (2 * h.fr + 1), 4);
  h.lds_obs = align_up(h.L.o_mt, 16) + ((h.mmax || h.kmax) ? h.map_bytes : h.map_bytes8) +
              4 * h.fv_words + align_up(h.dd, 16) + 4 * MFG_WAVE + h.dirt_cap / 8 +
              8 * (s->n_agents > MFG_WAVE ? 2 : 1) * h.dd +  // + per-window-cell agent masks (u64 per 64 agents)
              (h.dirt_cap ? 4 * h.dd : 0) +  // + window dirt map
              8 * MFG_WAVE +  // + packed-mode projection queue
              (h.maxpts == 0 || h.maxpts <= MFG_OBS_FLAT_MAXPTS ? 4 * h.dd : 0);  // + stashed tag words (FLAT)
  // replay kernel slice: [hdr 32 B][MT + perm (record bytes o_mt..o_perm+2nf, 16 B aligned)][shuffle tables]
  {
    h.xchg_ordered = v.shuffle_table_path ? 0 : probe_xchg_order(device);
    h.replay_mtperm = align_up(4 * 624 + 2 * h.nf, 16);  // o_perm == o_mt + 2496 (make_layout)
    h.replay_sink_off = 4 * RP_HDR_N + h.replay_mtperm;
    h.replay_stab_off = h.replay_sink_off + 2 * MFG_WAVE;  // u16 sinks (replay_shuffle, mt_twist)
    h.replay_stab_n = h.xchg_ordered ? RP_STAB_N : MFG_STAB_N;
    h.lds_replay_per_wave = align_up(h.replay_stab_off + 4 * h.replay_stab_n, 16);
    h.replay_top14 = h.nf < 16384 && !v.full_temper;  // (mfg_variant.full_temper: that path on small levels)
  }
  pcg64_seed(s->env_seed, &h.pcg_init_hi, &h.pcg_init_lo, &h.pcg_inc_hi, &h.pcg_inc_lo);
  // static tables
  std::vector<uint8_t> door_of(HW, 0xFF);
  for (int d = 0; d < s->n_doors; d++) door_of[s->door_cells[d]] = (uint8_t)d;
  std::vector<int16_t> cell_f(HW, -1);
  for (int f = 0; f < s->n_floor; f++) cell_f[s->floor_cells[f]] = (int16_t)f;
  std::vector<uint8_t> node_ok(s->n_floor ? s->n_floor : 1, 0);
  for (int f = 0; f < s->n_floor; f++) {
    const int c = s->floor_cells[f], x = c / s->W, y = c % s->W;
    for (int dx = -1; dx <= 1; dx++)
      for (int dy = -1; dy <= 1; dy++) {
        const int nx = x + dx, ny = y + dy;
        if ((dx || dy) && nx >= 0 && ny >= 0 && nx < s->H && ny < s->W && cell_f[nx * s->W + ny] >= 0) node_ok[f] = 1;
      }
  }
  std::vector<uint16_t> base_map(h.map_bytes / 2, 0);
  std::vector<uint8_t> base_map8(h.map_bytes8, 0);
  for (int c = 0; c < HW; c++)
    if (s->level[c] == 1) { base_map[c] = CM_WALL; base_map8[c] = CM_WALL; }
  std::vector<int32_t> wd;
  const int reach = h.fr;
  for (int k = 0; k < s->n_walls && k < s->n_doors; k++) {
    const int wc = s->wall_cells[k], dc = s->door_cells[k];
    const int dx = wc / s->W - dc / s->W, dy = wc % s->W - dc % s->W;
    if ((dx < 0 ? -dx : dx) <= 2 * reach && (dy < 0 ? -dy : dy) <= 2 * reach) {
      wd.push_back(k); wd.push_back(wc); wd.push_back(dc);
    }
  }
  h.n_wd_pairs = (int)(wd.size() / 3);
  h.max_pairs += h.n_wd_pairs;
  // LDS holds up to MFG_PAIRS_LDS pairs (the usual case); the bound's remainder spills to an HBM pool
  h.pairs_lds = std::min(h.max_pairs, MFG_PAIRS_LDS);
  if (v.pairs_lds > 0) h.pairs_lds = std::max(1, std::min(h.pairs_lds, (int)v.pairs_lds));  // mfg_variant
  h.lds_obs += 12 * h.pairs_lds;
  h.lds_obs_shared = align_up(h.L.o_mt, 16) + ((h.mmax || h.kmax) ? h.map_bytes : h.map_bytes8) + 12 * h.pairs_lds;
  h.lds_obs_wave = align_up(h.lds_obs - h.lds_obs_shared, 16);
  h.obs_slot_bytes = 0;
  if (!h.maxpts) {  // long-ray render: the per-agent tables go to an HBM pool slot per resident wave (k_obs_lr)
    h.obs_slot_bytes = align_up(h.lds_obs_wave, 256);
    h.lds_obs = h.lds_obs_shared;
    h.lds_obs_wave = 0;
  }
  if (h.lds_full > MFG_LDS_MAX || h.lds_obs > MFG_LDS_MAX || h.lds_replay_per_wave > MFG_LDS_MAX) {
    delete e; return fail("env record does not fit one CU's 160 KB of LDS");
  }
  std::vector<int8_t> rp((size_t)h.nrays * h.maxpts * 2, 0);
  std::vector<uint32_t> rp16((size_t)h.nrays * h.lrpts, 0u);  // long-ray render: dx & 0xFFFF | dy << 16
  std::vector<uint8_t> rlen(h.nrays);
  std::vector<uint64_t> rdiag(h.nrays, 0ull);
  for (int r = 0; r < h.nrays; r++) {
    const int p0 = s->ray_off[r], p1 = s->ray_off[r + 1];
    if (p1 - p0 > (h.maxpts ? h.maxpts : h.lrpts) || p1 - p0 > h.fr + 1) {
      delete e; return fail("ray longer than its radius + 1 points");
    }
    if (p1 - p0 < 1 || s->ray_pts[2 * p0] != 0 || s->ray_pts[2 * p0 + 1] != 0) {  // k_obs relies on it
      delete e; return fail("every ray must start at the origin (bresenham_loop, ray_caster.py:141-199)");
    }
    rlen[r] = (uint8_t)(p1 - p0);
    if (!h.maxpts) {  // (the long-ray walk tests diagonal steps from consecutive points itself)
      for (int p = p0; p < p1; p++)
        rp16[(size_t)r * h.lrpts + (p - p0)] =
            ((uint32_t)s->ray_pts[2 * p] & 0xFFFFu) | ((uint32_t)s->ray_pts[2 * p + 1] << 16);
      continue;
    }
    for (int p = p0 + 1; p < p1; p++)
      if (s->ray_pts[2 * p] != s->ray_pts[2 * p - 2] && s->ray_pts[2 * p + 1] != s->ray_pts[2 * p - 1])
        rdiag[r] |= 1ull << (p - p0);
    for (int p = p0; p < p1; p++) {
      rp[((size_t)r * h.maxpts + (p - p0)) * 2] = (int8_t)s->ray_pts[2 * p];
      rp[((size_t)r * h.maxpts + (p - p0)) * 2 + 1] = (int8_t)s->ray_pts[2 * p + 1];
    }
  }
  int rc = 0;
  rc |= upload(e, s->level, HW, &h.level);
  rc |= upload(e, door_of.data(), HW, &h.door_of);
  rc |= upload(e, s->wall_cells, s->n_walls, &h.wall_cells);
  rc |= upload(e, s->door_cells, s->n_doors, &h.door_cells);
  rc |= upload(e, s->floor_cells, s->n_floor, &h.floor_init);
  rc |= upload(e, rp.data(), rp.size(), &h.ray_pts);
  rc |= upload(e, rlen.data(), rlen.size(), &h.ray_len);
  rc |= upload(e, rdiag.data(), rdiag.size(), &h.ray_diag);
  h.ray_pts16 = nullptr;
  if (!h.maxpts) rc |= upload(e, rp16.data(), rp16.size(), &h.ray_pts16);
  {  // static light-blocking table per (origin floor cell, ray): walls only; door-dependent points flagged
    // (32-bit point masks: rays of up to 32 points; longer rays test every point against the cell map)
    const size_t n = (size_t)s->n_floor * h.nrays * 3;
    h.ray_static = nullptr;
    if (n * 4 <= ((size_t)256 << 20) && h.maxpts && h.maxpts <= 32) {
      std::vector<uint32_t> rs(n, 0u);
      auto wall = [&](int x, int y) { return x >= 0 && y >= 0 && x < s->H && y < s->W && s->level[x * s->W + y] == 1; };
      auto door = [&](int x, int y) { return x >= 0 && y >= 0 && x < s->H && y < s->W && door_of[x * s->W + y] != 0xFF; };
      for (int f = 0; f < s->n_floor; f++) {
        const int ox = s->floor_cells[f] / s->W, oy = s->floor_cells[f] % s->W;
        for (int r = 0; r < h.nrays; r++) {
          uint32_t* o = &rs[((size_t)f * h.nrays + r) * 3];
          for (int p = 0; p < rlen[r]; p++) {
            const int x = ox + rp[((size_t)r * h.maxpts + p) * 2], y = oy + rp[((size_t)r * h.maxpts + p) * 2 + 1];
            if (wall(x, y)) o[0] |= 1u << p;
            else if (door(x, y)) o[2] |= 1u << p;
            if (p > 0 && ((rdiag[r] >> p) & 1)) {
              const int px = ox + rp[((size_t)r * h.maxpts + p - 1) * 2], py = oy + rp[((size_t)r * h.maxpts + p - 1) * 2 + 1];
              const bool w1 = wall(x, py), w2 = wall(px, y), d1 = door(x, py), d2 = door(px, y);
              if (w1 && w2) o[1] |= 1u << p;
              else if ((w1 || d1) && (w2 || d2)) o[2] |= 1u << p;
            }
          }
        }
      }
      rc |= upload(e, rs.data(), rs.size(), &h.ray_static);
    }
  }
  rc |= upload(e, base_map.data(), base_map.size(), &h.base_map);
  rc |= upload(e, base_map8.data(), base_map8.size(), &h.base_map8);
  rc |= upload(e, cell_f.data(), cell_f.size(), &h.cell_f);
  {  // layer records (MfgLayerRec)
    std::vector<MfgLayerRec> lrec((size_t)h.A * h.lmax);
    std::vector<uint64_t> ab2((size_t)h.A * h.lmax, 0ull);
    for (int a = 0; a < h.A; a++)
      for (int l = 0; l < s->n_layers[a]; l++) {
        MfgLayerRec& R = lrec[(size_t)a * h.lmax + l];
        R = MfgLayerRec{0u, 0u, 0ull};
        const int kind = s->layers[a][l].kind, tag = s->layers[a][l].tag;
        if (kind == MFG_LAYER_TAG) {
          if (tag >= MFG_TAG_AGENT0 + MFG_WAVE) ab2[(size_t)a * h.lmax + l] = 1ull << (tag - MFG_TAG_AGENT0 - MFG_WAVE);
          else if (tag >= MFG_TAG_AGENT0) R.agent_bits = 1ull << (tag - MFG_TAG_AGENT0);
          else if (tag == MFG_TAG_DOORS) R.flags = LR_DOOR;
          else if (tag == MFG_TAG_DIRT) R.flags = LR_DIRT;
          else if (tag == MFG_TAG_MACHINES) R.flags = LR_MACHINE;
          else R.unit_tags = 1u << tag;
        } else if (kind == MFG_LAYER_COMBINED) {
          if (h.comb_fast[a]) {
            R.unit_tags = h.comb_unit_tags[a];
            R.agent_bits = h.comb_agents[a];
            ab2[(size_t)a * h.lmax + l] = h.comb_agents2[a];
          }
          else R.flags = LR_ORDERED;
        } else if (kind == MFG_LAYER_BATTERY) {
          R.flags = LR_BATTERY;
        } else if (kind == MFG_LAYER_GLOBALPOS) {
          R.flags = LR_GLOBALPOS;
        }
      }
    rc |= upload(e, lrec.data(), lrec.size(), &h.lrec);
    rc |= upload(e, ab2.data(), ab2.size(), &h.lrec_ab2);
  }
  rc |= upload(e, node_ok.data(), node_ok.size(), &h.node_ok);
  rc |= upload(e, wd.data(), wd.size(), &h.wd_pairs);
  if (rc) { delete e; return -1; }
  if (hipMalloc((void**)&e->d_spec, sizeof(MfgDevSpec)) != hipSuccess ||
      hipMemcpy(e->d_spec, &h, sizeof(MfgDevSpec), hipMemcpyHostToDevice) != hipSuccess) {
    delete e; return fail("spec upload failed");
  }
  if (hipMalloc((void**)&e->d_state, (size_t)h.L.size * (size_t)n_envs) != hipSuccess) {
    delete e; return fail("state allocation failed");
  }
  if (h.max_pairs > h.pairs_lds) {  // identifier-pair spill in HBM, one slice per env
    void* pool = nullptr;
    if (hipMalloc(&pool, (size_t)12 * (h.max_pairs - h.pairs_lds) * (size_t)n_envs) != hipSuccess) {
      delete e; return fail("pair pool allocation failed");
    }
    e->d_bufs.push_back(pool);
    h.pair_pool = (int*)pool;
  }
  {  // replay launch order (longest debt first): debt histogram, per-env bucket, env order
    void* p = nullptr;
    const size_t bytes = 4 * (size_t)RP_NB + (size_t)n_envs + 4 * ((size_t)n_envs + 4);
    if (hipMalloc(&p, bytes) != hipSuccess) {
      delete e; return fail("replay order allocation failed");
    }
    e->d_bufs.push_back(p);
    e->rp_hist = (int*)p;
    e->rp_order = (int*)p + RP_NB;
    e->rp_key = (uint8_t*)(e->rp_order + n_envs + 4);
  }
  {  // auto-reset done lists, both empty
    void* lst = nullptr;
    const size_t bytes = (size_t)2 * 4 * ((size_t)n_envs + 2);
    if (hipMalloc(&lst, bytes) != hipSuccess || hipMemset(lst, 0, bytes) != hipSuccess) {
      if (lst) (void)hipFree(lst);
      delete e; return fail("done list allocation failed");
    }
    e->d_bufs.push_back(lst);
    h.rd_list = (int32_t*)lst;
    void* fl = nullptr;
    if (hipMalloc(&fl, (size_t)n_envs) != hipSuccess || hipMemset(fl, 0, (size_t)n_envs) != hipSuccess) {
      if (fl) (void)hipFree(fl);
      delete e; return fail("done flag allocation failed");
    }
    e->d_bufs.push_back(fl);
    h.rd_flag = (uint8_t*)fl;
  }
  int prio_lo = 0, prio_hi = 0;  // the resets' stream first: their waves are a long serial chain each
  (void)hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
  if (hipStreamCreateWithPriority(&e->aux, hipStreamNonBlocking, prio_hi) != hipSuccess ||
      hipEventCreateWithFlags(&e->ev_fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&e->ev_join, hipEventDisableTiming) != hipSuccess) {
    delete e; return fail("stream/event creation failed");
  }
  if (h.bfs_bytes && !h.bfs_off) {  // BFS scratch in HBM, one slice per env
    void* pool = nullptr;
    if (hipMalloc(&pool, (size_t)h.bfs_bytes * (size_t)n_envs) != hipSuccess) {
      delete e; return fail("BFS scratch allocation failed");
    }
    e->d_bufs.push_back(pool);
    h.bfs_pool = (uint8_t*)pool;
  }
  if (hipMemcpy(e->d_spec, &h, sizeof(MfgDevSpec), hipMemcpyHostToDevice) != hipSuccess) {
    delete e; return fail("spec upload failed");
  }
  e->maxpts = h.maxpts;
  {  // k_resetdone's grid: the waves resident at once (one round; each strides over the done list)
    const int wpb = wpb_for(h.lds_full);
    int per_cu = 0, n_cu = 0;
    const hipError_t occ = h.lane_passes == 2 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_resetdone<2>, wpb * 64,
                                                                                 (size_t)h.lds_full * wpb)
                                     : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_resetdone<1>, wpb * 64,
                                                                                 (size_t)h.lds_full * wpb);
    if (occ != hipSuccess ||
        hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) {
      delete e; return fail("occupancy query failed");
    }
    e->rd_blocks = std::max(1, per_cu) * std::max(1, n_cu);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_replay_done, 64, (size_t)h.lds_replay_per_wave) !=
        hipSuccess) {
      delete e; return fail("occupancy query failed");
    }
    e->rpd_blocks = std::max(1, per_cu) * std::max(1, n_cu);
    e->n_cu = std::max(1, n_cu);
#ifndef MFG_REPLAY2
#define MFG_REPLAY2 1  // 0: never, 1: when the 1-wave replay slice leaves <= 2 waves per SIMD, 2: always
#endif
    e->replay2 = h.xchg_ordered && (size_t)h.lds_replay_per_wave + RP2_RING <= MFG_LDS_MAX &&
                 (MFG_REPLAY2 == 2 || (MFG_REPLAY2 == 1 && MFG_LDS_MAX / (size_t)h.lds_replay_per_wave <= 8));
    e->overlap = !v.serial &&  // mfg_variant.serial: one stream, for per-kernel attribution
                 (MFG_RESET_OVERLAP == 2 || (MFG_RESET_OVERLAP == 1 && (long long)h.A * h.nf >= 16384));
    // with long resets (overlap) and a rule that consumes the floor order inside a step, the envs that finish
    // or respawn dirt would otherwise pay up to K steps of debt on the critical path (C4: 6.7 -> 7.4M env-steps/s)
#ifndef MFG_REPLAY_EACH
#define MFG_REPLAY_EACH 0  // 1: the per-step replay beside the render for every overlapped spec, -1: never (timing)
#endif
    e->replay_each = MFG_REPLAY_EACH >= 0 && e->overlap && (h.step_rng || MFG_REPLAY_EACH);
    // render shape: one wave per env, or (ray length >= 10) one env per workgroup of nwv waves sharing the cell
    // map, whichever keeps more waves per CU (C5: 3 single-wave slices of 49 KB fit a CU, 2 workgroups of 4)
    {
      auto waves_per_cu = [&](int nwv) {
        const size_t wg = nwv == 1 ? (size_t)h.lds_obs : (size_t)h.lds_obs_shared + (size_t)nwv * h.lds_obs_wave;
        return (int)std::min<size_t>(32, (MFG_LDS_MAX / wg) * nwv);
      };
      int best = waves_per_cu(1);
      if (h.maxpts >= 10)
        for (int nwv : {2, 4, 8}) {
          const size_t wg = (size_t)h.lds_obs_shared + (size_t)nwv * h.lds_obs_wave;
          if (wg <= MFG_LDS_MAX && waves_per_cu(nwv) > best) { best = waves_per_cu(nwv); e->obs_nwv = nwv; }
        }
    }
    const int ow = std::min(MFG_WPB, wpb_for(h.lds_obs));
    const int obs_per_cu = std::max(1, std::min(32 / ow, (int)(MFG_LDS_MAX / ((size_t)h.lds_obs * ow))));
    e->obs_list_blocks = obs_per_cu * std::max(1, n_cu);
  }
  if (!h.maxpts) {  // long-ray render: one HBM pool slot per resident wave (one wave per SIMD)
    h.obs_slots = (int)std::max<long long>(1, std::min<long long>(n_envs, 4LL * e->n_cu));
    if (v.render_slots > 0) h.obs_slots = std::min(h.obs_slots, (int)v.render_slots);  // mfg_variant (tests)
    void* pool = nullptr;
    // two slot ranges: the done-list render on the second stream and the render of the other envs run concurrently
    if (hipMalloc(&pool, (size_t)h.obs_slot_bytes * (size_t)h.obs_slots * 2) != hipSuccess) {
      delete e; return fail("long-ray render pool allocation failed");
    }
    e->d_bufs.push_back(pool);
    h.obs_pool = (uint8_t*)pool;
    if (hipMemcpy(e->d_spec, &h, sizeof(MfgDevSpec), hipMemcpyHostToDevice) != hipSuccess) {
      delete e; return fail("spec upload failed");
    }
  }
  *out = e;
  return 0;
}

extern "C" int mfg_destroy(mfg_engine* e) {
  if (!e) return 0;
  DevGuard g(e->device);
  for (void* p : e->d_bufs) (void)hipFree(p);
  if (e->d_spec) (void)hipFree(e->d_spec);
  if (e->d_state) (void)hipFree(e->d_state);
  for (auto& m : e->marks) { e->ev_free.push_back(m.a); e->ev_free.push_back(m.b); }
  for (hipEvent_t ev : e->ev_free) (void)hipEventDestroy(ev);
  if (e->aux) (void)hipStreamSynchronize(e->aux);
  if (e->ev_fork) (void)hipEventDestroy(e->ev_fork);
  if (e->ev_join) (void)hipEventDestroy(e->ev_join);
  if (e->aux) (void)hipStreamDestroy(e->aux);
  delete e;
  return 0;
}

// record layout for host-side decoding (tests, snapshots):
// [size, o_hdr, ..., o_perm, lmax, obs_agent_stride, lds_full, xchg_ordered, o_machines, ..., scratch_bytes, o_logic,
//  reset_overlap (1: with auto-reset and obs, a step's resets and their render run on the engine's second stream)]
extern "C" int mfg_layout(const mfg_engine* e, int32_t* out) {
  const MfgLayout& L = e->h.L;
  const int32_t v[] = {L.size, L.o_hdr, L.o_rule_ctr, L.o_agent_pos, L.o_agent_arr, L.o_agent_par, L.o_frozen_org,
                       L.o_frozen_gp, L.o_door, L.o_items, L.o_pods, L.o_drops, L.o_dests, L.o_dirt_pos,
                       L.o_dirt_id, L.o_battery, L.o_frozen_bat, L.o_dirt_amt, L.o_pcg, L.o_mt, L.o_perm,
                       e->h.lmax, e->h.obs_agent_stride, e->h.lds_full, e->h.xchg_ordered, L.o_machines,
                       L.o_maints, L.o_mstate, L.o_mpath, L.o_grank, e->h.dirt_cap, e->h.lds_logic, e->h.lds_obs,
                       e->h.lds_replay_per_wave, e->h.bfs_off, e->h.bfs_bytes, e->h.max_pairs, e->h.scratch_bytes,
                       L.o_logic, e->overlap ? 1 : 0};
  const int n = (int)(sizeof(v) / sizeof(v[0]));
  for (int i = 0; i < n; i++) out[i] = v[i];
  return n;
}

extern "C" void* mfg_state_ptr(mfg_engine* e) { return e ? e->d_state : nullptr; }

// waves per workgroup for a per-wave LDS slice: up to MFG_WPB, as many as one CU's LDS holds
static int wpb_for(size_t lds) { return (int)std::max<size_t>(1, std::min<size_t>(MFG_WPB, MFG_LDS_MAX / std::max<size_t>(lds, 1))); }
static unsigned env_grid(const mfg_engine* e, int wpb) { return (unsigned)((e->B + wpb - 1) / wpb); }
// launch geometry of a kernel with `lds` bytes of dynamic LDS per wave
#define GEOM(lds) dim3(env_grid(e, wpb_for(lds))), dim3(wpb_for(lds) * 64), (size_t)(lds) * wpb_for(lds)
// waves per workgroup of k_logic / k_obs. k_logic runs one wave per workgroup (C3: 0.1544 -> 0.1507 ms; its slot
// frees as soon as its env is done); k_obs keeps 4 (1 and 2 measured within noise in round 2)
static const int obs_wpb = MFG_WPB, logic_wpb = 1;
#define GEOMW(lds, W) dim3(env_grid(e, std::min(W, wpb_for(lds)))), dim3(std::min(W, wpb_for(lds)) * 64), \
    (size_t)(lds) * std::min(W, wpb_for(lds))

// the render kernels are instantiated in mfg_obs_*.hip (launch_obs_inst, mfg_kernels.h)
template <int MP, typename OT, int PK>
static hipError_t launch_obs_t(mfg_engine* e, OT* obs, const ObsPacked& pk, hipStream_t st, const uint8_t* skip,
                               const int32_t* list) {
  ObsLaunch L;
  L.mw = e->obs_nwv > 1;
  if (MP == 0) {  // long-ray render: a resident grid, workgroup g owns HBM pool slot g (k_obs_lr)
    L.mw = false;
    L.W = 1;
    L.grid = (unsigned)e->h.obs_slots;
    L.lds = (size_t)e->h.lds_obs;
  } else if (L.mw) {  // one env per workgroup
    L.W = e->obs_nwv;
    L.lds = (size_t)e->h.lds_obs_shared + (size_t)L.W * e->h.lds_obs_wave;
    const long long per_cu = std::max<long long>(1, (long long)(MFG_LDS_MAX / L.lds));
    L.grid = list ? (unsigned)std::min<long long>(e->B, per_cu * e->n_cu) : (unsigned)e->B;
  } else {
    L.W = std::min(obs_wpb, wpb_for(e->h.lds_obs));
    L.grid = list ? (unsigned)std::min<long long>(env_grid(e, L.W), e->obs_list_blocks) : env_grid(e, L.W);
    L.lds = (size_t)e->h.lds_obs * L.W;
  }
  L.B = e->B;
  L.d_spec = e->d_spec;
  L.d_state = e->d_state;
  L.mm = e->h.mmax || e->h.kmax;
  L.dirt = e->h.dirt_cap != 0;
  return launch_obs_inst<MP, OT, PK>(L, obs, pk, st, skip, list);
}

#define DISPATCH_MP(MPVAL, CALL) \
  switch (MPVAL) {               \
    case 0: { constexpr int MP = 0; CALL; } break; \
    case 4: { constexpr int MP = 4; CALL; } break; \
    case 6: { constexpr int MP = 6; CALL; } break; \
    case 8: { constexpr int MP = 8; CALL; } break; \
    case 10: { constexpr int MP = 10; CALL; } break; \
    case 12: { constexpr int MP = 12; CALL; } break; \
    case 14: { constexpr int MP = 14; CALL; } break; \
    case 16: { constexpr int MP = 16; CALL; } break; \
    case 18: { constexpr int MP = 18; CALL; } break; \
    case 24: { constexpr int MP = 24; CALL; } break; \
    case 32: { constexpr int MP = 32; CALL; } break; \
    case 48: { constexpr int MP = 48; CALL; } break; \
    case 64: { constexpr int MP = 64; CALL; } break; \
    default: return fail("unsupported ray length"); \
  }

// check a packed-obs descriptor (host memory) against the engine: returns 0 or fails
static int check_packed(const mfg_engine* e, const mfg_packed_obs* p) {
  if (!p) return fail("MFG_OBS_PACKED needs an mfg_packed_obs descriptor");
  if ((p->idx == nullptr) != (p->val == nullptr)) return fail("packed obs: idx and val must both be set or both NULL");
  if (p->idx && p->cap <= 0) return fail("packed obs: cap must be > 0 when idx/val are given");
  if (p->emb && (p->emb_dim <= 0 || p->emb_dim > MFG_MAX_EMB || !p->wt))
    return fail("packed obs: emb needs wt and 0 < emb_dim <= MFG_MAX_EMB");
  if ((size_t)e->h.obs_agent_stride > 65535) return fail("packed obs: lmax*h*w >= 65536 does not fit the u16 idx");
  return 0;
}
// the k-th fused step's rows of a packed-obs descriptor
static ObsPacked packed_rows(const mfg_engine* e, const mfg_packed_obs* p, int k) {
  const size_t ba = (size_t)k * (size_t)e->B * (size_t)e->h.A;
  ObsPacked pk;
  pk.cap = p->idx ? p->cap : 0;
  pk.E = p->emb ? p->emb_dim : 0;
  pk.idx = p->idx ? p->idx + ba * pk.cap : nullptr;
  pk.val = p->val ? p->val + ba * pk.cap : nullptr;
  pk.cnt = p->count ? p->count + ba : nullptr;
  pk.wt = p->wt;
  pk.bias = p->bias;
  pk.emb = p->emb ? p->emb + ba * pk.E : nullptr;
  return pk;
}

// render obs of every env into obs (obs_dtype 0 = f32, 1 = f64, 2 = packed: obs -> mfg_packed_obs, row k)
static int launch_obs(mfg_engine* e, void* obs, int obs_dtype, hipStream_t st, int k = 0,
                      const uint8_t* skip = nullptr, const int32_t* list = nullptr, int kid = MFG_K_OBS) {
  hipError_t err = hipSuccess;
  PROF_BEGIN(e, st);
  ObsPacked none{};
  if (obs_dtype == MFG_OBS_PACKED) {
    const ObsPacked pk = packed_rows(e, (const mfg_packed_obs*)obs, k);
    // entries only (no projection registers: the render keeps its ray prefetch) or entries + fused obs_proj
    if (pk.emb) DISPATCH_MP(e->maxpts, err = (launch_obs_t<MP, float, 2>(e, (float*)nullptr, pk, st, skip, list)))
    else DISPATCH_MP(e->maxpts, err = (launch_obs_t<MP, float, 1>(e, (float*)nullptr, pk, st, skip, list)))
  } else if (obs_dtype == MFG_OBS_F64) {
    DISPATCH_MP(e->maxpts, err = (launch_obs_t<MP, double, 0>(e, (double*)obs, none, st, skip, list)));
  } else {
    DISPATCH_MP(e->maxpts, err = (launch_obs_t<MP, float, 0>(e, (float*)obs, none, st, skip, list)));
  }
  if (err != hipSuccess) return fail(std::string("k_obs launch: ") + hipGetErrorString(err));
  PROF_END(e, st, kid);
  return 0;
}

// reset (init=1: create envs, seeding env i with random.seed(seed_base + i)); obs_dtype 0=f32 1=f64.
// With a mask only the masked envs are reset, but obs (if given) is rendered for every env.
static int reset_impl(mfg_engine* e, const uint8_t* mask, void* obs, int obs_dtype, int init, uint64_t seed_base,
                      void* stream);
extern "C" int mfg_reset(mfg_engine* e, const uint8_t* mask, void* obs, int obs_dtype, int init,
                         uint64_t seed_base, void* stream) {
  ENGINE_CALL(e, reset_impl(e, mask, obs, obs_dtype, init, seed_base, stream));
}
static int reset_impl(mfg_engine* e, const uint8_t* mask, void* obs, int obs_dtype, int init, uint64_t seed_base,
                      void* stream) {
  if (obs && obs_dtype != MFG_OBS_F32 && obs_dtype != MFG_OBS_F64 && obs_dtype != MFG_OBS_PACKED)
    return fail("obs_dtype must be MFG_OBS_F32, MFG_OBS_F64 or MFG_OBS_PACKED");
  if (obs && obs_dtype == MFG_OBS_PACKED && check_packed(e, (const mfg_packed_obs*)obs)) return -1;
  hipStream_t st = (hipStream_t)stream;
  PROF_BEGIN(e, st);
  if (e->h.lane_passes == 2)
    hipLaunchKernelGGL(k_reset<2>, GEOM(e->h.lds_full), st, e->d_spec, e->d_state, (long long)e->B, mask, init,
                       (unsigned long long)seed_base);
  else
    hipLaunchKernelGGL(k_reset<1>, GEOM(e->h.lds_full), st, e->d_spec, e->d_state, (long long)e->B, mask, init,
                       (unsigned long long)seed_base);
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) return fail(std::string("k_reset launch: ") + hipGetErrorString(err));
  PROF_END(e, st, MFG_K_RESET);
  return obs ? launch_obs(e, obs, obs_dtype, st) : 0;
}

// Pay all pending floor-shuffle debt (membership-only shuffles of the reference's move checks, Q3).
static int replay_impl(mfg_engine* e, void* stream);
extern "C" int mfg_replay(mfg_engine* e, void* stream) { ENGINE_CALL(e, replay_impl(e, stream)); }
static int replay_impl(mfg_engine* e, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  PROF_BEGIN(e, st);
  // one wave per workgroup: a workgroup's slot is held until its slowest env's debt is paid and debts differ
  // per env, so single-wave workgroups free each slot as soon as its env is done (C3: 11.17 -> 10.91 ms per
  // K=8 launch against 4 waves per workgroup)
  // longest debt first (C3: 10.95 -> 10.47 ms per K=8 launch, the order kernels included)
  const unsigned g256 = (unsigned)((e->B + 255) / 256);
  {
    HIPCHK(hipMemsetAsync(e->rp_hist, 0, 4 * RP_NB, st));
    hipLaunchKernelGGL(k_rp_count, dim3(g256), dim3(256), 0, st, e->d_spec, e->d_state, (long long)e->B, e->rp_hist,
                       e->rp_key);
    hipLaunchKernelGGL(k_rp_scan, dim3(1), dim3(RP_NB), 0, st, e->rp_hist);
    hipLaunchKernelGGL(k_rp_place, dim3(g256), dim3(256), 0, st, (long long)e->B, e->rp_hist, e->rp_key,
                       e->rp_order);
  }
  if (e->replay2)  // large floor lists: a producer and a consumer wave per env (replay_env2)
    hipLaunchKernelGGL(k_replay2, dim3((unsigned)e->B), dim3(2 * MFG_WAVE),
                       (size_t)e->h.lds_replay_per_wave + RP2_RING, st, e->d_spec, e->d_state, (long long)e->B,
                       (const int*)e->rp_order);
  else {
    size_t lds = (size_t)e->h.lds_replay_per_wave;
#ifdef MFG_RP_LDS_W
    // measurement only (tools/gpu_r05a.sh, DESIGN §4 "k_replay, round 5"): the same kernel with its LDS slice padded so
    // that at most MFG_RP_LDS_W waves per SIMD fit, for the occupancy curve
    lds = std::max(lds, (size_t)((MFG_LDS_MAX / (4 * MFG_RP_LDS_W)) & ~15));
#endif
    hipLaunchKernelGGL(k_replay, dim3((unsigned)e->B), dim3(64), lds, st, e->d_spec, e->d_state, (long long)e->B,
                       (const int*)e->rp_order);
  }
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) return fail(std::string("k_replay launch: ") + hipGetErrorString(err));
  PROF_END(e, st, MFG_K_REPLAY);
  return 0;
}

// K steps. actions: device [K][B][A] int32, or NULL -> Philox4x32-10 synthetic actions keyed
// (philox_seed, env_base+env) at counter (step_base+k, agent). Outputs (each may be NULL):
// reward [K][B][A] f64, done [K][B] u8, obs [K][B][A][lmax][d][d], ev_act/ev_watch [K][B][A] u8,
// ev_misc [K][B][MFG_EV_MISC_N] i32. auto_reset: envs that finish are reset (the obs row is then the first
// observation of the new episode). Per step: k_logic, k_resetdone (auto_reset), k_obs (obs); then one
// k_replay for the whole call.
static int step_impl(mfg_engine* e, int K, const int32_t* actions, uint32_t philox_seed, uint32_t env_base,
                     int64_t step_base, double* reward, uint8_t* done, void* obs, int obs_dtype, uint8_t* ev_act,
                     uint8_t* ev_watch, int32_t* ev_misc, int auto_reset, void* stream);
extern "C" int mfg_step(mfg_engine* e, int K, const int32_t* actions, uint32_t philox_seed, uint32_t env_base,
                        int64_t step_base, double* reward, uint8_t* done, void* obs, int obs_dtype,
                        uint8_t* ev_act, uint8_t* ev_watch, int32_t* ev_misc, int auto_reset, void* stream) {
  ENGINE_CALL(e, step_impl(e, K, actions, philox_seed, env_base, step_base, reward, done, obs, obs_dtype, ev_act,
                           ev_watch, ev_misc, auto_reset, stream));
}
static int step_impl(mfg_engine* e, int K, const int32_t* actions, uint32_t philox_seed, uint32_t env_base,
                     int64_t step_base, double* reward, uint8_t* done, void* obs, int obs_dtype, uint8_t* ev_act,
                     uint8_t* ev_watch, int32_t* ev_misc, int auto_reset, void* stream) {
  if (K < 1) return fail("K must be >= 1");
  if (auto_reset & ~(MFG_STEP_AUTO_RESET | MFG_STEP_DEFER_REPLAY)) return fail("unknown mfg_step flag bits");
  const bool defer = (auto_reset & MFG_STEP_DEFER_REPLAY) != 0;  // the call's final replay left for a later call
  auto_reset &= MFG_STEP_AUTO_RESET;
  if (obs && obs_dtype != MFG_OBS_F32 && obs_dtype != MFG_OBS_F64 && obs_dtype != MFG_OBS_PACKED)
    return fail("obs_dtype must be MFG_OBS_F32, MFG_OBS_F64 or MFG_OBS_PACKED");
  if (obs && obs_dtype == MFG_OBS_PACKED && check_packed(e, (const mfg_packed_obs*)obs)) return -1;
  hipStream_t st = (hipStream_t)stream;
  const size_t B = (size_t)e->B, A = (size_t)e->h.A;
  const size_t obs_row = B * A * (size_t)e->h.obs_agent_stride * (obs_dtype == MFG_OBS_F64 ? 8 : 4);
  for (int k = 0; k < K; k++) {
    const size_t kb = (size_t)k * B;
    if (e->h.respawn_mask && !e->replay_each) {
      PROF_BEGIN(e, st);
      hipLaunchKernelGGL(k_replay_sel, dim3((unsigned)e->B), dim3(64), (size_t)e->h.lds_replay_per_wave, st, e->d_spec,
                         e->d_state, (long long)e->B);
      hipError_t err = hipGetLastError();
      if (err != hipSuccess) return fail(std::string("k_replay_sel launch: ") + hipGetErrorString(err));
      PROF_END(e, st, MFG_K_REPLAY_SEL);
    }
    {
    PROF_BEGIN(e, st);
    // k_logic<FULL, MAINT, SEL, NW> over every env (NW: 64-lane agent / door passes, MfgDevSpec::nw)
#define LAUNCH_LOGIC(FULL, MAINT, SEL, LDS)                                                                        \
  do {                                                                                                             \
    if (e->h.lane_passes == 2)                                                                                              \
      hipLaunchKernelGGL((k_logic<FULL, MAINT, SEL, 2>), GEOMW(LDS, logic_wpb), st, e->d_spec, e->d_state,         \
                         (long long)e->B, act_k, philox_seed, env_base, (long long)(step_base + k), rew_k, done_k, \
                         eva_k, evw_k, evm_k, auto_reset, e->rd_slot);                                             \
    else                                                                                                           \
      hipLaunchKernelGGL((k_logic<FULL, MAINT, SEL, 1>), GEOMW(LDS, logic_wpb), st, e->d_spec, e->d_state,         \
                         (long long)e->B, act_k, philox_seed, env_base, (long long)(step_base + k), rew_k, done_k, \
                         eva_k, evw_k, evm_k, auto_reset, e->rd_slot);                                             \
  } while (0)
    const int32_t* act_k = actions ? actions + kb * A : nullptr;
    double* rew_k = reward ? reward + kb * A : nullptr;
    uint8_t* done_k = done ? done + kb : nullptr;
    uint8_t* eva_k = ev_act ? ev_act + kb * A : nullptr;
    uint8_t* evw_k = ev_watch ? ev_watch + kb * A : nullptr;
    int32_t* evm_k = ev_misc ? ev_misc + kb * MFG_EV_MISC : nullptr;
    const int cnt_lds = 4 * MFG_WAVE * e->h.lane_passes;  // per-door count scratch after the staged prefix
    if (e->h.bfs_bytes) {
      // maintainers: the envs where no maintainer re-routes (and no dirt spawn fires) this step run with the step
      // prefix + maintainer state/paths staged (no MT, permutation or BFS scratch: several times the occupancy), the
      // rest with the full record
      const int ms0 = e->h.L.o_mstate & ~15;
      const int lm_lds = e->h.L.o_logic + (((e->h.L.o_mpath + 15) & ~15) - ms0) + cnt_lds;
      LAUNCH_LOGIC(true, true, 1, lm_lds);
      LAUNCH_LOGIC(true, true, 2, e->h.lds_logic);
    } else if (e->h.step_rng) {
      // RespawnDirt is the only in-step RNG consumer here: the envs without a spawn this step run the lean step at
      // its occupancy, the few with one (C4 ~1/16) the full-record step
      const int lean_lds = e->h.L.o_logic + cnt_lds;
      LAUNCH_LOGIC(false, false, 1, lean_lds);
      LAUNCH_LOGIC(true, false, 2, e->h.lds_logic);
    } else {
      LAUNCH_LOGIC(false, false, 0, e->h.lds_logic);
    }
#undef LAUNCH_LOGIC
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) return fail(std::string("k_logic launch: ") + hipGetErrorString(err));
    PROF_END(e, st, MFG_K_LOGIC);
    }
    const int rd_cur = e->rd_slot;
    e->rd_slot ^= 1;  // the next k_logic appends to the other list (and empties this one after k_resetdone)
    void* obs_k = obs && obs_dtype != MFG_OBS_PACKED ? (void*)((uint8_t*)obs + (size_t)k * obs_row) : obs;
    // With auto-reset and obs, the done envs are reset and rendered on the engine's second stream while the
    // caller's stream renders every other env (k_logic's rd_flag tells k_obs which to leave out): a step's
    // resets are a few hundred latency-bound waves (C4: ~2.4 ms) that the full render hides.
    const bool split = e->overlap && auto_reset && obs_k;
    // the per-step replay (replay_each): on the second stream after the resets, beside the render when split (the
    // render reads the step prefix and cell map, the replay writes MT / permutation and two header words the
    // render does not read; the next step's k_logic waits for both streams)
    const bool replay_now = e->replay_each && k + 1 < K;
    if (replay_now && !split && replay_impl(e, stream)) return -1;
    hipStream_t rs = split ? e->aux : st;
    if (split) {
      HIPCHK(hipEventRecord(e->ev_fork, st));
      HIPCHK(hipStreamWaitEvent(e->aux, e->ev_fork, 0));
    }
    if (auto_reset) {
      PROF_BEGIN(e, rs);
      // the done envs' debt first, at k_replay's occupancy; k_resetdone then finds none left to pay
      hipLaunchKernelGGL(k_replay_done, dim3((unsigned)std::min<long long>(e->B, e->rpd_blocks)), dim3(64),
                         (size_t)e->h.lds_replay_per_wave, rs, e->d_spec, e->d_state, (long long)e->B, rd_cur);
      const int wpb = wpb_for(e->h.lds_full);
      const long long nwg = std::min<long long>(env_grid(e, wpb), e->rd_blocks);
      if (e->h.lane_passes == 2)
        hipLaunchKernelGGL(k_resetdone<2>, dim3((unsigned)nwg), dim3(wpb * 64), (size_t)e->h.lds_full * wpb, rs,
                           e->d_spec, e->d_state, (long long)e->B, rd_cur);
      else
        hipLaunchKernelGGL(k_resetdone<1>, dim3((unsigned)nwg), dim3(wpb * 64), (size_t)e->h.lds_full * wpb, rs,
                           e->d_spec, e->d_state, (long long)e->B, rd_cur);
      hipError_t err = hipGetLastError();
      if (err != hipSuccess) return fail(std::string("k_resetdone launch: ") + hipGetErrorString(err));
      PROF_END(e, rs, MFG_K_RESETDONE);
    }
    if (split) {
      const int32_t* lst = e->h.rd_list + (size_t)rd_cur * (size_t)(e->B + 2);
      if (launch_obs(e, obs_k, obs_dtype, rs, k, nullptr, lst, MFG_K_OBS_DONE)) return -1;
      if (replay_now && replay_impl(e, rs)) return -1;
    }
    if (split) {
      if (launch_obs(e, obs_k, obs_dtype, st, k, e->h.rd_flag, nullptr, MFG_K_OBS)) return -1;
    } else if (obs_k && launch_obs(e, obs_k, obs_dtype, st, k)) {
      return -1;
    }
    if (split) {
      HIPCHK(hipEventRecord(e->ev_join, e->aux));
      HIPCHK(hipStreamWaitEvent(st, e->ev_join, 0));
    }
  }
  return defer ? 0 : replay_impl(e, stream);
}

// snapshots (checkpoints == fixtures): whole state buffer device<->device, B * layout.size bytes
static int copy_state(mfg_engine* e, void* dst, const void* src, void* stream) {
  if (!dst || !src) return fail("null argument");
  HIPCHK(hipMemcpyAsync(dst, src, (size_t)e->h.L.size * e->B, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return 0;
}
extern "C" int mfg_export_state(mfg_engine* e, void* dst, void* stream) {
  ENGINE_CALL(e, copy_state(e, dst, e->d_state, stream));
}
extern "C" int mfg_import_state(mfg_engine* e, const void* src, void* stream) {
  ENGINE_CALL(e, copy_state(e, e->d_state, src, stream));
}
extern "C" int mfg_profile(mfg_engine* e, int enable) {
  if (!e) return fail("null engine");
  e->prof = enable != 0;
  return 0;
}

static int profile_read_impl(mfg_engine* e, double* total_ms, int64_t* launches, int n);
extern "C" int mfg_profile_read(mfg_engine* e, double* total_ms, int64_t* launches, int n) {
  ENGINE_CALL(e, profile_read_impl(e, total_ms, launches, n));
}
static int profile_read_impl(mfg_engine* e, double* total_ms, int64_t* launches, int n) {
  if (!total_ms || !launches) return fail("null argument");
  for (int k = 0; k < n; k++) { total_ms[k] = 0.0; launches[k] = 0; }
  for (const auto& m : e->marks) HIPCHK(hipEventSynchronize(m.b));  // marks may sit on both streams
  for (const auto& m : e->marks) {
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, m.a, m.b));
    if (m.k < n) { total_ms[m.k] += ms; launches[m.k] += 1; }
    e->ev_free.push_back(m.a);
    e->ev_free.push_back(m.b);
  }
  e->marks.clear();
  return 0;
}

extern "C" int64_t mfg_state_bytes(const mfg_engine* e) { return e ? (int64_t)e->h.L.size * e->B : -1; }
extern "C" int mfg_abi_version(void) { return MFG_ABI_VERSION; }

// Measured HBM peak for the bench's roofline (mfg.h mfg_hbm_copy): one 16-B non-temporal load + store per lane, one
// lane per 16 B (tools/copy_probe.hip on the MI355X, 2 GiB: this form 6.58 TB/s of read + write bytes; plain 6.24;
// 4-8 per lane unrolled 5.6-6.0; grid-stride loops 4.7-4.9; hipMemcpy 5.0; torch copy_ 4.5)
typedef unsigned mfg_v4u __attribute__((ext_vector_type(4)));
static __global__ void __launch_bounds__(256) k_hbm_copy(mfg_v4u* __restrict__ dst, const mfg_v4u* __restrict__ src,
                                                         long long n16) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n16) __builtin_nontemporal_store(__builtin_nontemporal_load(&src[i]), &dst[i]);
}
extern "C" int mfg_hbm_copy(void* dst, const void* src, int64_t nbytes, void* stream) {
  if (!dst || !src || nbytes <= 0 || (nbytes & 15) || (((uintptr_t)dst | (uintptr_t)src) & 15))
    return fail("mfg_hbm_copy: null pointer, or size/alignment not a multiple of 16 B");
  const long long n16 = (long long)(nbytes >> 4);
  if ((n16 + 255) / 256 > 0x7fffffffLL) return fail("mfg_hbm_copy: size too large");
  hipLaunchKernelGGL(k_hbm_copy, dim3((unsigned)((n16 + 255) / 256)), dim3(256), 0, (hipStream_t)stream, (mfg_v4u*)dst,
                     (const mfg_v4u*)src, n16);
  HIPCHK(hipGetLastError());
  return 0;
}
