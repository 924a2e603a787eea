/*
 * tcmp.h -- C-ABI of the MI355X torque-constrained RRT* engine (libtcmp.so).
 *
 * Plain pointers and sizes only: every array argument is a HOST pointer owned by the caller,
 * row-major, fp64 configurations (7 per row), int32/int64 counts.  Every entry point returns
 * an int status (0 = ok, < 0 = error; tcmp_last_error() gives a thread-local message).
 * Calls are synchronous (the engine's stream is drained before return) unless noted.
 *
 * Each entry point names the reference interface it replaces
 * (HIRO-group/torque_constrained_motion_planning @ v0, src/...).
 */
#ifndef TCMP_H_
#define TCMP_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct tcmp_handle tcmp_handle;
typedef struct tcmp_comm tcmp_comm;  /* multi-GPU communicator (tcmp_dist_init, below) */

/* torque_test modes, panda_primitives.py:228-236 */
#define TCMP_TORQUE_BASE 0 /* get_torque_limits_not_exceded_test_base   panda_primitives.py:13 */
#define TCMP_TORQUE_NOV 1  /* get_torque_limits_not_exceded_test_v3_nov panda_primitives.py:118 */
#define TCMP_TORQUE_RNE 2  /* get_torque_limits_not_exceded_test_v4     panda_primitives.py:155 */
#define TCMP_TORQUE_DYN 3  /* get_torque_limits_not_exceded_test_v2     panda_primitives.py:60
                              (M, C, g from rne.py's model: the reference's pdm is not shipped) */

/* plan status codes (tcmp_plan_result.status) */
#define TCMP_PLAN_OK 0            /* path found and validated (rrt_star.py:211) */
#define TCMP_PLAN_START_GOAL_COLLISION 1 /* rrt_star.py:152-154 */
#define TCMP_PLAN_NO_GOAL 2       /* rrt_star.py:199-201 */
#define TCMP_PLAN_VALIDATION_FAILED 3 /* rrt_star.py:208-210 */
#define TCMP_PLAN_MINJERK_ASSERT 4 /* min_jerk_v2.py:166 num_intervals == 0 */

/* ---- lifetime -------------------------------------------------------------------------- */
int tcmp_create(int device, tcmp_handle** out);
int tcmp_destroy(tcmp_handle* h);
const char* tcmp_last_error(void);
int tcmp_device_count(int* n);
int tcmp_version(void);
/* wait for all work queued on the handle's HIP stream */
int tcmp_synchronize(tcmp_handle* h);
/* profiling builds (-DTCMP_PROF) only: k_edges clock breakdown accumulated since create
 * (total, work fetch, collision, torque, bookkeeping, tier-4 exact, ...) and exact-test
 * outcome counts and mesh-stage clocks (12..35, then 44..51), the nearest scan's clocks and
 * visit counts (36..43), n <= 52; zeros otherwise. */
int tcmp_debug_counters(tcmp_handle* h, uint64_t* out, int32_t n);

/* Peak microbenchmarks on the handle's device (the spec peaks are re-measured
 * before use): out[0] fp64 vector FMA TFLOP/s, out[1] fp32 packed (v_pk_fma_f32) TFLOP/s,
 * out[2] HBM GB/s of a 1 GiB float4 device copy (read + write bytes), out[3] 0.  Best of five
 * launches each; allocates 2 GiB for the copy while it runs.  No reference counterpart. */
int tcmp_microbench(tcmp_handle* h, double* out);

/* Fixed obstacles (replaces Problem.fixed bodies + pybullet getClosestPoints,
 * utils.py:3165-3218 / 2833-2849).  n_obs oriented boxes, 15 doubles each:
 * centre(3), rotation R (9, row-major, columns = box axes, world frame), half extents(3). */
int tcmp_set_scene(tcmp_handle* h, const double* obb, int32_t n_obs);

/* Fixed convex-mesh obstacles (replaces pybullet GEOM_MESH bodies in Problem.fixed: Bullet
 * collides the convex hull of the mesh vertices, utils.py:2833-2880, closest points with
 * distance = -0.04).  All in the world frame; n_mesh hulls, rows of mesh m are
 * [off[m], off[m+1]) of each array (offsets start at 0):
 *   verts  V x 3            hull vertices
 *   planes F x 4            facet planes n.x <= d (unit outward n, d = max n.v)
 *   edges  E x 4 (int32)    hull edges: va vb (mesh-local vertex rows) f1 f2 (mesh-local
 *                           plane rows of the two adjacent facets)
 *   boxes  n_mesh x 18      outer box containing the hull: centre(3), R(9, columns = axes),
 *                           half(3); then the half extents (3) of a box with the same centre
 *                           and axes inside the hull (zeros = none)
 * Replaces the previous mesh set; boxes from tcmp_set_scene are kept (and vice versa).
 * Host-side hull construction: torque_constrained_motion_planning_amd/hull.py. */
int tcmp_set_meshes(tcmp_handle* h, const double* verts, const int32_t* vert_off,
                    const double* planes, const int32_t* plane_off, const int32_t* edges,
                    const int32_t* edge_off, const double* boxes, int32_t n_mesh);

/* A set of n hulls in tcmp_set_meshes' layout (world frame, rows [off[m], off[m+1])). */
typedef struct tcmp_hulls {
  const double* verts;        /* V x 3 */
  const int32_t* vert_off;    /* n + 1 */
  const double* planes;       /* F x 4: unit outward n, d */
  const int32_t* plane_off;
  const int32_t* edges;       /* E x 4: va vb f1 f2 (hull-local rows) */
  const int32_t* edge_off;
} tcmp_hulls;

/* Optional level-of-detail hulls for the current meshes (same count, call after
 * tcmp_set_meshes): inner[m] must lie inside mesh m's hull and outer[m] must contain it.
 * The kernels use them only as certificates before the exact test ("free" when the outer
 * hulls' depth is below 0.04 - 1e-4, "collision" when the inner hulls' depth exceeds
 * 0.04 + 1e-4), so results do not depend on them -- only speed.  hull.py builds them. */
int tcmp_set_mesh_lods(tcmp_handle* h, const tcmp_hulls* inner, const tcmp_hulls* outer,
                       int32_t n_mesh);

/* Optional inscribed spheres for the current meshes (call after tcmp_set_meshes; cleared by
 * it): spheres[n_mesh][k][4] = (cx, cy, cz, r), world frame, each ball inside mesh m's hull
 * (checked against the stored facet planes, n.c + r <= d + 1e-9; status -1 otherwise);
 * k must be 16.  Like the LODs they are certificates only (same reference semantics,
 * utils.py:2833 closest points at -0.04): a link sphere and a mesh sphere overlapping by
 * >= 0.04 + 1e-4 prove "collision", and the full hulls' projections on the direction between
 * the most-overlapping pair's centres overlapping by < 0.04 - 1e-4 prove "free".  Results do
 * not depend on them -- only speed.  spheres.py builds them. */
int tcmp_set_mesh_spheres(tcmp_handle* h, const double* spheres, int32_t n_mesh, int32_t k);

/* Self-collision (get_collision_fn(..., self_collisions=True), utils.py:3165-3191 with the
 * pairs of get_self_link_pairs, utils.py:3125-3149): enable != 0 adds the 33 link pairs of
 * the arm whose moving-ancestor joint sets differ and that are not parent/child (link0 is the
 * base, outside get_links; link8 has no geometry), same -0.04 closest-point threshold
 * (pairwise_link_collision -> get_closest_points default, utils.py:2781,2833,2851).  Every
 * later collision check (configs, edges, planning rounds, rewiring) includes them.  Off by
 * default, as in the reference planner (SELF_COLLISIONS = False, utils.py:56). */
int tcmp_set_self_collision(tcmp_handle* h, int32_t enable);

/* per-kernel-family device timing of plans (tcmp_plan_result.ms_*: hipEvents recorded around
 * each family, event nodes inside captured round graphs).  On by default; off records no
 * events, so a round graph holds kernel nodes only and ms_* stay 0 (queries run concurrently
 * on several engines, whose event spans would include each other's kernels anyway).  No
 * reference counterpart (instrumentation). */
int tcmp_set_timing(tcmp_handle* h, int32_t enable);

/* ---- batched physics (host arrays in/out) ---------------------------------------------- */
/* rne(q, qd, qdd) with add_payload(r, m) state made explicit: payload iff payload_mass > 0
 * (rne.py:181-254).  q, qd, qdd, tau: n x 7. */
int tcmp_rne_batch(tcmp_handle* h, const double* q, const double* qd, const double* qdd,
                   int64_t n, double payload_mass, double* tau);

/* torque test on n configurations (panda_primitives.py:13-193); qd/qdd may be NULL (zeros,
 * the search-time call torque_fn(q)).  ok: n int32 (1 = within limits). */
int tcmp_torque_ok(tcmp_handle* h, const double* q, const double* qd, const double* qdd,
                   int64_t n, int32_t torque_mode, double payload_mass, int32_t* ok);

/* collision_fn(q) on n configurations (utils.py:3165-3218): joint limits then every moving
 * link hull vs every obstacle, penetration >= 0.04 m.  collides: n int32. */
int tcmp_check_configs(tcmp_handle* h, const double* q, int64_t n, int32_t* collides);

/* Body-level check any(pairwise_collision(robot, b) for b in obstacles) on n configurations
 * (franka_ik_fast.py:78, panda_primitives.py:260 -> utils.py:2872-2880 body_collision ->
 * get_closest_points(max_distance=-0.04), :2833): every link of the robot body, i.e. the moving
 * links AND the static base panda_link0, penetration >= 0.04 m, no joint-limit test.
 * collides: n int32. */
int tcmp_check_body(tcmp_handle* h, const double* q, int64_t n, int32_t* collides);

/* Penetration depth of the static base panda_link0 (world = base frame) against each obstacle
 * of the scene: the tcmp_set_scene boxes, then the tcmp_set_meshes meshes (n must be their
 * sum).  The q-independent half of tcmp_check_body. */
int tcmp_base_pd(tcmp_handle* h, double* pd, int32_t n);

/* safe_path_force_aware(extend(from, to), collision, torque) for n edges (rrt_star.py:90-98,
 * utils.py:3068-3077 with the given resolution vector (7, NULL = 0.1 as the planner uses)).
 * n_safe = len(safe prefix), n_steps = len(extend), last = prefix[-1] (valid if n_safe>0). */
int tcmp_check_edges(tcmp_handle* h, const double* from, const double* to, int64_t n,
                     const double* resolutions, int32_t torque_mode, double payload_mass,
                     int32_t* n_safe, int32_t* n_steps, double* last);

/* argmin over tree nodes of the weighted distance (rrt_star.py:9-14,171), first index wins
 * ties.  tree: T x 7, samples: n x 7, weights: 7 positive (NULL = 10 = 1/radius).  Runs the
 * planner's own nearest path: the radix-tree cell index of the tree and the pruned exact
 * scan k_nearest_wave32 (fp32 first pass, fp64 decision). */
int tcmp_nearest(tcmp_handle* h, const double* tree, int64_t T, const double* samples,
                 int64_t n, const double* weights, int32_t* idx);

/* dynam_fn min-jerk sampling (panda_primitives.py:299-316 -> min_jerk_v2.py:80-222):
 * n_wp waypoints (7 each), ni samples per segment; q/qd/qdd: (n_wp-1)*ni x 7. */
int tcmp_minjerk(tcmp_handle* h, const double* waypoints, int64_t n_wp, int64_t ni, double* q,
                 double* qd, double* qdd);

/* final validation loop (rrt_star.py:208-210) + Conf.torques (utils.py:3376-3377, rne
 * without payload).  first_fail = index of the first failing sample or -1.  tau may be NULL. */
int tcmp_validate_traj(tcmp_handle* h, const double* q, const double* qd, const double* qdd,
                       int64_t n, int32_t torque_mode, double payload_mass, int64_t* first_fail,
                       double* tau);

/* ---- goal IK ------------------------------------------------------------ */
/* ikfast get_ik (ikfast_panda_arm.cpp:12839 -> ComputeIk :12770, free joint = joint7 :398),
 * batched: poses n x 12 = panda_link8 in panda_link0 (rotation 9 row-major, then position 3,
 * the eerot/eetrans of :12854-12862), free_q7 n values.  sols: n x 8 x 7 (the count[i]
 * solutions of row i packed first, angles in (-pi, pi]); count: n.  Joint limits are NOT
 * applied (the reference filters afterwards, ikfast.py:166). */
int tcmp_ik(tcmp_handle* h, const double* poses, const double* free_q7, int64_t n, double* sols,
            int32_t* count);

/* ikfast get_fk (ikfast_panda_arm.cpp:12907 -> ComputeFk :307): q n x 7 -> poses n x 12. */
int tcmp_fk(tcmp_handle* h, const double* q, int64_t n, double* poses);

/* ---- the RRT* engine (rrt_star_force_aware, rrt_star.py:151-211) ------------------------ */
typedef struct {
  double start[7];
  double goal[7];
  double weights[7];      /* distance weights, 1/radius (panda_primitives.py:333-334) */
  double resolutions[7];  /* extend resolutions (panda_primitives.py:337: radius) */
  double radius;          /* rewire radius ([0.01], panda_primitives.py:346) */
  double goal_probability;/* 0.2 (rrt_star.py:151) */
  double goal_tolerance;  /* 1e-2 (rrt_star.py:178) */
  double payload_mass;    /* Problem.payload_mass (torque tests) */
  double execution_time;  /* Problem.execution_time (dynam_fn) */
  uint64_t seed;          /* Philox4x32-10 key for device sampling */
  int64_t max_nodes;      /* tree capacity (>= samples + 1) */
  int32_t max_batch;      /* largest round size that will be used */
  int32_t torque_mode;
} tcmp_plan_cfg;

typedef struct {
  int32_t status;         /* TCMP_PLAN_* */
  int32_t goal_found;
  int64_t n_nodes;
  int64_t n_samples;
  int64_t goal_node;
  int64_t n_waypoints;    /* len(goal_n.retrace()) */
  int64_t n_traj;         /* min-jerk samples */
  int64_t first_fail;
  uint64_t edge_steps;    /* extend steps checked (the new edges', then the rewire edges') */
  uint64_t pairs_tested;  /* link x obstacle pair classifications */
  uint64_t pairs_sat;     /* pairs reaching the OBB SAT tier */
  uint64_t pairs_exact;   /* exact hull tests */
  uint64_t nn_pairs;      /* (candidate, node) distance evaluations */
  double ms_nearest;      /* summed device time per kernel family (hipEvents) */
  double ms_edges;
  double ms_insert;
  double ms_rewire;
  double ms_finish;
  int64_t launches_nearest;
  uint64_t nn_box_tests;  /* (candidate, chunk-box) lower-bound tests of the pruned scan */
  double ms_nn_scan;      /* the k_nearest_wave32 launches alone (part of ms_nearest) */
  uint64_t snap_sum;      /* sum over rounds of the snapshot size T_r */
  uint64_t nn_full_pairs; /* sum over rounds of T_r * B_r: the brute-force scan's pair count */
  int64_t launches_nn_scan; /* k_nearest_wave32 launches (a one-node first round needs none) */
  uint64_t n_rewires;     /* new.rewire(n, d, path[:-1]) calls (rrt_star.py:187-192) on this
                             engine's lanes */
  uint64_t rewire_steps;  /* the rewire edges' extend steps (part of edge_steps, not k_edges') */
  int64_t graph_launches; /* tcmp_plan_run calls of this plan replayed as one captured graph */
  int64_t fused_plans;    /* plans of the fused rounds this plan grew in (tcmp_plan_run_fused;
                             0: its own rounds).  The fleet's kernel times (ms_*) are reported
                             on its first engine, every plan counts the fleet's rounds */
  double ms_edge_prep;    /* the edge order's sort and work records before k_edges (ms_edges
                             times k_edges alone) */
  double goal_cost;       /* goal_n.cost (rrt_star.py:25-27: the path's summed distance fn)
                             when a goal node exists, else 0 */
  int64_t goal_depth;     /* edges root -> goal node (len(retrace nodes) - 1), else 0 */
} tcmp_plan_result;

/* start a query: checks collision(start), collision(goal) (rrt_star.py:152), allocates the
 * tree and inserts the root.  result->status is set (0 or START_GOAL_COLLISION). */
int tcmp_plan_begin(tcmp_handle* h, const tcmp_plan_cfg* cfg, tcmp_plan_result* result);

/* one round of nb candidates.  samples == NULL: device Philox sampling (batched frontier,
 * at most one goal-biased lane per round).  Otherwise samples (nb x 7) and is_goal (nb) are
 * the host's draws (nb = 1 reproduces the reference loop exactly).  goal_found (nullable)
 * is written after a stream sync; pass NULL to keep rounds asynchronous. */
int tcmp_plan_round(tcmp_handle* h, const double* samples, const uint8_t* is_goal, int32_t nb,
                    int32_t* goal_found);

/* shared-tree rounds (SURVEY 8e's alternative to replica trees): every rank of `c` has the
 * same open plan (tcmp_plan_begin with identical cfg; max_nodes for the whole tree,
 * max_batch >= ceil(batch / world)) and calls this with the same n_samples / batch; rank r
 * takes lanes [r B / W, (r + 1) B / W) of each round of B and the ranks exchange, per round,
 * the goal lane and the accepted-edge counts (RCCL all-reduce / all-gather on the engine
 * stream) and then their new node records (one group of in-place ncclBroadcast calls), so
 * every rank holds the tree a single engine builds with tcmp_plan_run(h, n_samples, batch).
 * World 1 is tcmp_plan_run. */
int tcmp_plan_run_shared(tcmp_handle* h, tcmp_comm* c, int64_t n_samples, int32_t batch);

/* the same rounds driven by one process over n engines (devices may repeat), the exchanges
 * done through host copies and device-to-device copies: the single-process form of
 * tcmp_plan_run_shared (and its parity check on one GPU). */
int tcmp_plan_run_group(tcmp_handle* const* hs, int32_t n, int64_t n_samples, int32_t batch);

/* fused multi-plan rounds: n (1..31) engines on one device, each with its own open plan (its
 * own scene, start, goal, seed), all at the same round, grow their trees together -- one set
 * of kernel launches per round serves every plan's lanes (tcmp_fleet.h), on hs[0]'s stream;
 * the other engines' streams are ordered before and after it.  Every plan's tree is
 * bit-identical to what tcmp_plan_run(hs[q], n_samples, batch) grows alone; finish and fetch
 * each plan on its own engine as usual.  Box scenes may differ per plan; a fleet over convex
 * meshes or with self-collision pairs must be ONE scene (every plan's the lead's: replica trees
 * of one query), otherwise the call returns -1.  The plans must share the distance weights, at
 * most ~330 box obstacles over all plans (the fused edge kernel's LDS), and fewer than 2^31
 * node / lane slots over the fleet.  The multi-query form of tcmp_plan_run
 * (collect_data.py:74-85 plans several start/goal queries per scene step). */
int tcmp_plan_run_fused(tcmp_handle* const* hs, int32_t n, int64_t n_samples, int32_t batch);

/* tcmp_plan_begin / tcmp_plan_finish on n engines (cfgs[q], results[q] for hs[q]): every
 * engine's work is queued first, then the host waits once per engine -- a fleet's begins and
 * finishes cost about one device round trip instead of n.  Same results as the one-engine
 * calls; the first failing engine's error is reported (its index in the message). */
int tcmp_plan_begin_many(tcmp_handle* const* hs, int32_t n, const tcmp_plan_cfg* cfgs,
                         tcmp_plan_result* results);
int tcmp_plan_finish_many(tcmp_handle* const* hs, int32_t n, tcmp_plan_result* results);

/* goal node of the open plan (-1 while none) and its cost -- goal_n.cost, the bound of the
 * informed rejection test (rrt_star.py:163-165); cost may be NULL. */
int tcmp_plan_goal(tcmp_handle* h, int64_t* node, double* cost);

/* device-sampled rounds of `batch` lanes until n_samples samples were drawn. */
int tcmp_plan_run(tcmp_handle* h, int64_t n_samples, int32_t batch);

/* retrace + dynam_fn min-jerk + final torque validation (rrt_star.py:199-211); fills result. */
int tcmp_plan_finish(tcmp_handle* h, tcmp_plan_result* result);

/* retrace only (rrt_star.py:199-200, goal_n.retrace()): the finish for a caller whose own
 * dynam_fn turns the waypoints into the trajectory (rrt_star.py:202 with a foreign dynam_fn).
 * No min-jerk, no validation: status is 0 (goal found) or TCMP_PLAN_NO_GOAL, n_traj 0,
 * first_fail -1; tcmp_plan_fetch then copies the waypoints. */
int tcmp_plan_retrace(tcmp_handle* h, tcmp_plan_result* result);

/* copy the finished plan: waypoints (n_waypoints x 7), trajectory q/qd/qdd (n_traj x 7),
 * psg (n_traj), tau = Conf.torques without payload (n_traj x 7).  Any pointer may be NULL. */
int tcmp_plan_fetch(tcmp_handle* h, double* waypoints, double* q, double* qd, double* qdd,
                    double* psg, double* tau);

/* digest of the open plan's tree, computed on the device: the sum over nodes i of a 64-bit
 * splitmix64 chain over (i, the node's 7 configuration and cost bits, its parent index), mod
 * 2^64 (torque_constrained_motion_planning_amd/shard.py tree_digest restates it).  Equal trees
 * give equal digests, so ranks of a shared-tree run (tcmp_plan_run_shared) can prove they hold
 * one tree by all-gathering it; n_nodes = the tree's node count. */
int tcmp_plan_digest(tcmp_handle* h, uint64_t* digest, int64_t* n_nodes);

/* debug: tree snapshot (cfg n x 7, cost n, parent n). */
int tcmp_plan_tree(tcmp_handle* h, int64_t cap, double* cfg, double* cost, int32_t* parent,
                   int64_t* n);

/* debug: the last round's nearest-neighbour step (rrt_star.py:171 for every lane): its nb
 * candidates (cand nb x 7), the chosen nearest node of each (nn, an index into the tree) and
 * the exact fp64 score of that node (sum_k (s_k - n_k)^2 when the weights are uniform, else
 * sum_k w_k (s_k - n_k)^2); snap = the snapshot size the round searched (nodes [0, snap)).
 * The first min(cap, nb) rows are copied; any array pointer may be NULL. */
int tcmp_plan_debug_round(tcmp_handle* h, int64_t cap, double* cand, int32_t* nn,
                          double* score, int64_t* snap, int32_t* nb);

/* ---- multi-GPU: query sharding + RCCL gather of solved paths -------------- */
/* One process per GPU; independent queries are dealt to ranks (collect_data.py:74-85 plans
 * them in a loop); the only collective is the gather of solved trajectories to rank 0.
 * A trajectory row is [q(7) qd(7) qdd(7) dt(1)] (Conf values / velocities / accelerations /
 * dt of create_trajectory, utils.py:3340-3347). */
#define TCMP_TRAJ_COLS 22
#define TCMP_REDUCE_SUM 0
#define TCMP_REDUCE_MAX 1

/* TCP rendezvous: rank 0 listens on addr:port; every other rank connects (retrying until
 * timeout_ms) and introduces itself with the job's identity (TCMP_JOB_ID, else the launcher's
 * TORCHELASTIC_RUN_ID, hashed with world and port: a stale or concurrent job is turned away).
 * Rank 0 sends its nbytes `blob` only after all world - 1 ranks have arrived; on a timeout it
 * closes every connection, so every rank fails together.  Host only, no GPU.  Used for the
 * ncclUniqueId; world == 1 returns at once. */
int tcmp_rendezvous(int32_t rank, int32_t world, const char* addr, int32_t port, void* blob,
                    int32_t nbytes, int32_t timeout_ms);

/* communicator of `world` ranks over RCCL on HIP device `device` (rank 0's unique id through
 * tcmp_rendezvous at addr:port).  world == 1: no RCCL communicator, no GPU touched. */
int tcmp_dist_init(int32_t rank, int32_t world, int32_t device, const char* addr, int32_t port,
                   tcmp_comm** out);
int tcmp_dist_destroy(tcmp_comm* c);
int tcmp_dist_rank(const tcmp_comm* c, int32_t* rank, int32_t* world);
/* ranks of the communicator's RCCL handle (ncclCommCount); 0 for a one-rank job, which has
 * no RCCL communicator.  Lets a multi-GPU run prove which collective world it ran in. */
int tcmp_dist_rccl_ranks(const tcmp_comm* c, int32_t* n);
/* device-synchronise this rank, then an RCCL all-reduce as the barrier */
int tcmp_dist_barrier(tcmp_comm* c);
/* in-place all-reduce of n doubles (op TCMP_REDUCE_SUM / TCMP_REDUCE_MAX) */
int tcmp_dist_allreduce(tcmp_comm* c, double* v, int32_t n, int32_t op);
/* all-gather of n int64 per rank: out = world x n, rank order */
int tcmp_dist_allgather_i64(tcmp_comm* c, const int64_t* in, int32_t n, int64_t* out);

/* gather every rank's solved paths to rank 0 (ncclGroupStart; ncclSend/ncclRecv;
 * ncclGroupEnd).  In: n_local paths, ids[i], rows[i], data = the paths' rows concatenated
 * (sum(rows) x TCMP_TRAJ_COLS); sizes = world x 2 int64 (queries, rows) of every rank when the
 * caller has all-gathered them already (tcmp_dist_allgather_i64), else NULL and the call does
 * the size all-gather itself.  Out, rank 0 only: n_queries paths in rank order (out_ids,
 * out_rows) with their rows concatenated in out_data, laid out by tcmp_gather_layout;
 * elsewhere n_queries = n_rows = 0.  Capacities too small: status -4 with n_queries / n_rows
 * set (the collective still completes on every rank).  Collective: every rank must call it.
 * Replaces the reference's host loop over queries (collect_data.py:74-85). */
int tcmp_gather_paths(tcmp_comm* c, int32_t n_local, const int64_t* ids, const int64_t* rows,
                      const double* data, const int64_t* sizes, int64_t cap_queries,
                      int64_t cap_rows, int64_t* out_ids, int64_t* out_rows, double* out_data,
                      int64_t* n_queries, int64_t* n_rows);

/* The two host-side halves of tcmp_gather_paths around its transport (RCCL send/recv on the
 * GPU; any byte transport works the same way).
 * tcmp_gather_pack: one rank's wire form -- hdr (2 n_local int64: id, rows of each path) and
 * body (sum(rows) x 22 doubles, the paths' rows concatenated; body may alias data).
 * tcmp_gather_unpack (rank 0): hdr_all / body_all hold every rank's wire form at the offsets of
 * tcmp_gather_layout(world, sizes); each rank's header rows are checked against the rows it
 * announced in sizes (status -6 otherwise: a transport that lost, duplicated or misplaced part
 * of a message), then the outputs are written as tcmp_gather_paths writes them (status -4
 * when the capacities are too small, n_queries / n_rows set).  Host only, no GPU. */
int tcmp_gather_pack(int32_t n_local, const int64_t* ids, const int64_t* rows, const double* data,
                     int64_t* hdr, double* body);
int tcmp_gather_unpack(int32_t world, const int64_t* sizes, const int64_t* hdr_all,
                       const double* body_all, int64_t cap_queries, int64_t cap_rows,
                       int64_t* out_ids, int64_t* out_rows, double* out_data, int64_t* n_queries,
                       int64_t* n_rows);

/* rank 0's receive layout of tcmp_gather_paths, host only: from sizes (world x 2: queries,
 * rows per rank) each rank's first header row q_off[k] and first trajectory row r_off[k] in
 * the rank-ordered output, and the totals.  Any output pointer may be NULL. */
int tcmp_gather_layout(int32_t world, const int64_t* sizes, int64_t* q_off, int64_t* r_off,
                       int64_t* total_q, int64_t* total_r);

#ifdef __cplusplus
}
#endif
#endif
