/*
 * vk_kinetics.h -- C ABI of the MI355X batched agent-kinetics engine.
 *
 * Drop-in boundary for the per-agent hot path of CovertLab/Lens ("vivarium").
 * The reference has no native FFI for this path: it is pure Python calling
 * numpy/scipy.  Each entry point below replaces one reference call site; the
 * Python host layer (lens_amd/native.py via ctypes) is the only caller.  See
 * INTEGRATION.md for the binding a vivarium maintainer would add.
 *
 *   vk_table_create / vk_table_destroy
 *       replaces KineticFluxModel.__init__ -> make_configuration /
 *       make_rate_laws (vivarium/library/kinetic_rate_laws.py:262-275,
 *       :43-98, :183-237).  The host compiler (lens_amd/rate_law_compiler.py)
 *       flattens the closures into the index arrays of vk_table_desc.
 *   vk_rate_fluxes
 *       replaces KineticFluxModel.get_fluxes (kinetic_rate_laws.py:277-297).
 *   vk_step_euler
 *       replaces ConvenienceKinetics.next_update
 *       (vivarium/processes/convenience_kinetics.py:303-352): one forward-Euler
 *       step, integer exchange counts truncated toward zero (:331).
 *   vk_step_dopri5
 *       replaces the reference's scipy.integrate.odeint step
 *       (vivarium/processes/Kremling2007_transport.py:384) for convenience
 *       networks: adaptive Dormand-Prince 5(4) over [0, dt] on the augmented
 *       system (internal species + per-reaction flux integrals).
 *   vk_field_uniform + vk_diffuse
 *       replace DiffusionField.diffuse / diffusion_delta
 *       (vivarium/processes/diffusion_field.py:385-407): fixed dt=0.01
 *       substeps of the reflect-boundary 5-point Laplacian, uniform-field skip.
 *   vk_gather
 *       replaces DiffusionField.get_local_environments (:362-379).
 *   vk_exchange_sorted / vk_exchange_atomic
 *       replace update_field_with_exchange (vivarium/core/registry.py:149-183)
 *       applied once per agent by Store.apply_update.
 *   vk_bin_sites
 *       replaces get_bin_site (vivarium/library/lattice_utils.py:18-40).
 *
 * Conventions
 *   - All array arguments are DEVICE pointers except vk_table_desc's, which are
 *     host pointers copied at vk_table_create.  The library never frees caller
 *     memory; vk_table is the only object it owns.
 *   - Agent arrays are structure-of-arrays with row stride `ld` (>= n_agents):
 *     element (row, agent) lives at [row * ld + agent].
 *   - Every call is asynchronous on `stream` (a hipStream_t; NULL = legacy
 *     default stream) and returns a vk_status.  Per-agent problems are
 *     reported in the caller's int32 status[] array (vk_agent_status bits).
 *   - All arithmetic is FP64.
 */
#ifndef VK_KINETICS_H
#define VK_KINETICS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VK_ABI_VERSION 1

typedef void *vk_stream_t;        /* hipStream_t */
typedef struct vk_table vk_table; /* opaque, device-resident reaction table */

enum vk_status {
    VK_OK = 0,
    VK_ERR_ARG = 1,   /* bad argument (null pointer, negative size, ...) */
    VK_ERR_HIP = 2,   /* a HIP runtime call failed; see vk_last_error() */
    VK_ERR_LIMIT = 3, /* network too large for the requested kernel variant */
    VK_ERR_NOMEM = 4
};

enum vk_agent_status {
    VK_AGENT_OK = 0,
    VK_AGENT_MAX_STEPS = 1,   /* integrator hit max_steps before t = dt */
    VK_AGENT_H_UNDERFLOW = 2, /* step size fell below 1e-14 * dt */
    VK_AGENT_NONFINITE = 4    /* NaN/Inf in the state or an exchange count */
};

/* Flattened rate-law table (lens_amd/rate_law_compiler.py:RateLawTable). */
typedef struct vk_table_desc {
    int32_t n_species;   /* rows of the agent concentration array            */
    int32_t n_dyn;       /* rows [0, n_dyn) receive deltas (non-external)    */
    int32_t n_reactions; /* flux rows                                        */
    int32_t n_rate_laws; /* (reaction, enzyme) closures, get_fluxes order    */
    int32_t n_params;    /* per-agent parameter rows (kcat, Km)              */
    int32_t n_ext;       /* exchange-count rows (external molecules)         */
    int32_t n_sets;      /* cofactor / partition sets                        */
    int32_t n_members;   /* (species, Km slot) members of all sets           */
    int32_t n_upd;       /* stoichiometry entries of dyn species             */
    int32_t n_exch;      /* stoichiometry entries of external molecules      */
    const int32_t *rl_reaction; /* [n_rate_laws] reaction row               */
    const int32_t *rl_enzyme;   /* [n_rate_laws] species row of the enzyme  */
    const int32_t *rl_kcat;     /* [n_rate_laws] parameter row of kcat_f    */
    const int32_t *rl_num_ptr;  /* [n_rate_laws+1] numerator sets           */
    const int32_t *rl_den_ptr;  /* [n_rate_laws+1] partition sets           */
    const int32_t *set_ptr;     /* [n_sets+1] members                       */
    const int32_t *mem_species; /* [n_members] species row                  */
    const int32_t *mem_param;   /* [n_members] parameter row of the Km      */
    const int32_t *upd_ptr;     /* [n_dyn+1]                                */
    const int32_t *upd_rxn;     /* [n_upd]                                  */
    const double *upd_coeff;    /* [n_upd]                                  */
    const int32_t *ex_ptr;      /* [n_ext+1]                                */
    const int32_t *ex_rxn;      /* [n_exch]                                 */
    const double *ex_coeff;     /* [n_exch]                                 */
} vk_table_desc;

typedef struct vk_ode_opts {
    double rtol;       /* relative tolerance (scipy RK45 semantics)          */
    double atol;       /* absolute tolerance                                 */
    int32_t max_steps; /* attempted steps per agent per call                 */
    int32_t variant;   /* 0 = agent-per-thread, table walked at run time
                              (n_dyn + n_reactions <= 32);
                          1 = agent-per-wavefront: one 64-lane wave per agent,
                              wave-reduced error norm, wave-uniform step
                              control (n_dyn + n_reactions <= 512);
                          2 = agent-per-thread, network-specialised
                              (vk_table_specialize);
                          3 = agent-per-wavefront, network-specialised:
                              rate laws padded to one shape per round of 64
                              lanes, per-lane operands in VGPRs
                              (vk_table_specialize with a wavefront source) */
} vk_ode_opts;

int vk_abi_version(void);
const char *vk_last_error(void);

int vk_table_create(const vk_table_desc *desc, vk_table **out);
int vk_table_destroy(vk_table *table);

/* Attach a network-specialised integrator to the table: `source` is the HIP
 * source lens_amd/codegen.py generates from the same table, compiled with
 * hiprtc for gfx950.  It defines `vk_dopri5_spec` (agent per lane: straight-
 * line rate laws, every species/parameter/stage value in VGPRs; used for
 * opts->variant == 2), `vk_dopri5_wspec` (agent per wavefront; variant 3),
 * or both. */
int vk_table_specialize(vk_table *table, const char *source);

/* flux[r*ld + a] = sum over the reaction's rate laws (exact reference order). */
int vk_rate_fluxes(const vk_table *t, int64_t n_agents, int64_t ld,
                   const double *params, const double *conc, double *flux,
                   vk_stream_t stream);

/* One reference Euler step.  If delta is NULL, conc rows [0, n_dyn) are
 * updated in place (conc += delta, the accumulate updater); otherwise conc is
 * left untouched and delta[s*ld+a] receives the reference's update value
 * (0 + sum_j (coeff_j*flux)*dt).  flux[r*ld+a] (set);
 * counts[e*ld+a] = sum_j trunc(((coeff_j*flux)*dt)*m2c[a]).               */
int vk_step_euler(const vk_table *t, int64_t n_agents, int64_t ld, double dt,
                  const double *params, double *conc, const double *mmol_to_counts,
                  double *delta, double *flux, int64_t *counts, int32_t *status,
                  vk_stream_t stream);

/* Adaptive Dormand-Prince 5(4) over [0, dt].  External/enzyme rows are held.
 * delta as for vk_step_euler (NULL: integrate conc in place; else
 * delta = y(dt) - y(0), conc untouched).  h_state[a]: step-size carry-over
 * (in/out; <= 0 selects the initial step).  flux = integral(flux)/dt;
 * counts from the integral; nsteps = attempted steps.                     */
int vk_step_dopri5(const vk_table *t, int64_t n_agents, int64_t ld, double dt,
                   const vk_ode_opts *opts, const double *params, double *conc,
                   const double *mmol_to_counts, double *delta, double *h_state,
                   double *flux, int64_t *counts, int32_t *status, int32_t *nsteps,
                   vk_stream_t stream);

/* vk_step_dopri5 (variant 2, after vk_table_specialize) fused with the
 * gather of the NEXT step's local environment: once agent a is integrated,
 * conc[map_row[i] * ld + a] = fields[map_field[i] * field_stride + bin_lin[a]]
 * for i < n_map (<= 8) -- the values vk_gather writes when it runs right after
 * the kinetics (DiffusionField.get_local_environments, diffusion_field.py:
 * 362-379, feeding ConvenienceKinetics.next_update, convenience_kinetics.py:
 * 303-352, one step later).  One launch and one sweep of the field lines
 * instead of two.                                                          */
int vk_step_dopri5_gather(const vk_table *t, int64_t n_agents, int64_t ld, double dt,
                          const vk_ode_opts *opts, const double *params, double *conc,
                          const double *mmol_to_counts, double *h_state, double *flux,
                          int64_t *counts, int32_t *status, int32_t *nsteps,
                          const double *fields, int64_t field_stride, const int32_t *bin_lin,
                          const int32_t *map_field, const int32_t *map_row, int32_t n_map,
                          vk_stream_t stream);

/* n_steps consecutive agent-steps of dt in one launch, for colonies whose
 * agents do not couple between steps (held externals; BASELINE config 2):
 * every step is vk_step_dopri5 variant 2's, bit for bit, with the state kept
 * in registers between steps.  Step s writes its mean fluxes at flux + s *
 * step_flux, its exchange counts at counts + s * step_counts and its attempts
 * at nsteps + s * step_nsteps (rows of ld, as vk_step_dopri5); conc and
 * h_state hold the end state, status ORs every step's bits.  Needs
 * vk_table_specialize with an agent-per-lane source.  Not a reference
 * interface: the reference steps agents one Delta t at a time
 * (Experiment.update, experiment.py:1351-1450).                            */
int vk_step_dopri5_multi(const vk_table *t, int64_t n_agents, int64_t ld, double dt, int32_t n_steps,
                         const vk_ode_opts *opts, const double *params, double *conc, const double *m2c,
                         double *h_state, double *flux, int64_t step_flux, int64_t *counts,
                         int64_t step_counts, int32_t *status, int32_t *nsteps, int64_t step_nsteps,
                         vk_stream_t stream);

/* Lattice fields: n_fields planes of rows x ny doubles, plane stride
 * field_stride.  Local rows may include halo rows of neighbouring ranks.   */

/* Uniform-plane test over rows [row_lo, row_hi) (diffusion_field.py:401-404).
 * summary[2f] == summary[2f+1] iff plane f holds a single value (both then
 * hold it); otherwise summary = (-inf, +inf) (a NaN plane is non-uniform).
 * Element-wise min of [2f] / max of [2f+1] over ranks gives the global test.
 * A non-uniform plane costs one 16-KiB chunk per probe block.              */
#define VK_UNIFORM_BLOCKS 512   /* scratch: n_fields * VK_UNIFORM_BLOCKS int32 */
int vk_field_uniform(const double *fields, int32_t n_fields, int64_t field_stride,
                     int32_t ny, int32_t row_lo, int32_t row_hi, double *summary,
                     int32_t *scratch, vk_stream_t stream);

/* Substeps [sub_begin, sub_begin+sub_count) of an n_sub-substep diffusion.
 * Substep j reads src(j) and writes dst(j):
 *   src(0) = field, src(j) = work[(j-1)&1]; dst(j) = work[j&1] except the
 *   last substep, which writes field = field + (new - field).
 * Owned rows are [row_lo, row_hi).  Within the call, substep j computes rows
 * [max(lo_min, row_lo-g), min(hi_max, row_hi+g)) with
 * g = sub_begin+sub_count-1-j (halo shrinking); rows lo_min and hi_max-1 are
 * reflected (Neumann) if they are global edges (edge_top/edge_bot != 0).
 * coeff_dt = (D/(dx*dy)) * 0.01.  uniform (nullable, a vk_field_uniform summary)
 * skips uniform planes.                                                      */
int vk_diffuse(double *field, double *work0, double *work1, int32_t n_fields,
               int64_t field_stride, int32_t ny, int32_t row_lo, int32_t row_hi,
               int32_t lo_min, int32_t hi_max, int32_t edge_top, int32_t edge_bot,
               int32_t sub_begin, int32_t sub_count, int32_t n_sub, double coeff_dt,
               const double *uniform, vk_stream_t stream);

/* vk_diffuse for one part of a row band's block (multi-GPU C4), so that the
 * halo exchange can run while the band computes what does not need it:
 *   VK_PART_INTERIOR  the first m = interior_passes passes of the block on the
 *                     rows whose inputs at the block's start are all owned
 *                     (10 (p+1) rows in from each side with halo rows, pass p);
 *   VK_PART_EDGES     the rest of those m passes (the rows next to the halo),
 *                     then the block's remaining passes whole;
 *   VK_PART_ALL       = vk_diffuse.
 * interior_passes <= 0 or > the block's passes means all of them.  INTERIOR
 * then EDGES (the halo in place before EDGES) equals vk_diffuse bit for bit.
 * Only the 10-deep plan (vk_set_stencil_depth(10), a block of 10 k substeps)
 * of a band of more than 2 * sub_count owned rows splits; otherwise
 * VK_ERR_LIMIT (nothing launched).  Replaces the same reference call as
 * vk_diffuse (diffusion_field.py:385-407).                                 */
enum { VK_PART_ALL = 0, VK_PART_INTERIOR = 1, VK_PART_EDGES = 2 };
int vk_diffuse_part(double *field, double *work0, double *work1, int32_t n_fields,
                    int64_t field_stride, int32_t ny, int32_t row_lo, int32_t row_hi,
                    int32_t lo_min, int32_t hi_max, int32_t edge_top, int32_t edge_bot,
                    int32_t sub_begin, int32_t sub_count, int32_t n_sub, double coeff_dt,
                    const double *uniform, int32_t part, int32_t interior_passes,
                    vk_stream_t stream);

/* As vk_diffuse for a call that ends at the last substep, except that the
 * last substep writes delta = new - field into `delta` (same layout; zero on
 * uniform planes) and leaves `field` as it was: DiffusionField.next_update's
 * delta (diffusion_field.py:385-394), for an accumulate updater that applies
 * it later (multi-rate schedules, lens_amd.process.BatchedDiffusionField).  */
int vk_diffuse_delta(double *field, double *work0, double *work1, double *delta, int32_t n_fields,
                     int64_t field_stride, int32_t ny, int32_t row_lo, int32_t row_hi, int32_t lo_min,
                     int32_t hi_max, int32_t edge_top, int32_t edge_bot, int32_t sub_begin,
                     int32_t sub_count, int32_t n_sub, double coeff_dt, const double *uniform,
                     vk_stream_t stream);

/* One whole-plane step of n_sub substeps (rows [0, rows), both edges
 * reflected) with the agent coupling carried by its passes -- one launch per
 * pass instead of vk_gather + the passes + vk_exchange_sorted, same results:
 *   - the first pass, before it changes anything, sets
 *       conc[gather_row[f]*conc_ld + a] = plane f at bin_lin[a]   (vk_gather)
 *   - the final pass, after writing plane f, adds
 *       counts[count_row[f]*counts_ld + a] / binvol_avogadro * 1000
 *     for the agents of each bin in agent order             (vk_exchange_sorted)
 * gather_row / count_row: host arrays of n_fields rows (-1 = none).  Agents
 * must be stored in bin order (bin_lin ascending, Colony.sort_by_bin), and
 * seg[r*nseg + s] (nseg = (ny+15)/16) = the first agent whose bin_lin >= r*ny + 16 s.
 * Uniform planes (the vk_field_uniform summary in `uniform`, nullable) keep
 * their values and still gather and exchange.  Returns VK_ERR_LIMIT and launches
 * nothing unless the step is planned as two or more pair-sum passes (the
 * tolerance mode, vk_set_stencil_mode(1), with kernel variants 20 / 70 and pass
 * depths 3..11; n_fields <= 8): the caller then runs the three steps itself.
 * Not a reference interface: DiffusionField.next_update (diffusion_field.py:
 * 362-407) and the agents' exchange updates (registry.py:149-183) fused.     */
int vk_diffuse_coupled(double *field, double *work0, double *work1, int32_t n_fields,
                       int64_t field_stride, int32_t ny, int32_t rows, int32_t n_sub, double coeff_dt,
                       const double *uniform, const int32_t *bin_lin, const int32_t *seg, int32_t nseg,
                       int64_t n_agents, const int32_t *gather_row, double *conc, int64_t conc_ld,
                       const int32_t *count_row, const int64_t *counts, int64_t counts_ld,
                       double binvol_avogadro, vk_stream_t stream);

/* Maximum substeps fused per HBM pass by vk_diffuse (temporal blocking; odd,
 * 1..15; 1 = one launch per substep; or 10, the default: a block of a multiple
 * of 10 substeps as 10-deep passes -- in the tolerance mode over three buffers
 * when the block ends the step, in the exact mode with the final pass re-reading
 * the step-start field -- and every other call at depth 9).  Odd depths plan
 * each call as the fewest odd-depth passes <= k, as even as possible.  Returns
 * the previous value; other k only query.  Exact mode: bit-identical for every
 * depth.                                                                    */
int vk_set_stencil_depth(int32_t k);

/* Fused-pass kernel variant.  Exact mode: 2 / 3 = wave tile with DPP lane
 * shifts, stage q lagging q rows (two live rows per stage), 3 / 6 rows
 * prefetched; 6 = variant 3 with streaming (non-temporal) stores (the exact
 * mode's kernel for 6 and 20-22).  Tolerance mode: 20 = pair-sum passes,
 * (W+N)+(S+E) with each pair added once and used by two cells, 3 FP64 ops
 * per cell-substep (default); 21 / 22 = 20 with 2 / 6 rows prefetched; 6 =
 * the 4-op FMA form.  Other values are ignored (retired variants 0, 1, 4, 5,
 * 7-16).  rows = output rows per tile (8..4096; 0 = auto from
 * the band height; other values keep the current).  Returns the previous
 * variant.  Tuning only: exact-mode results are bit-identical for every
 * setting; tolerance-mode results stay within 1e-13 of them.               */
int vk_set_stencil_kernel(int32_t variant, int32_t rows);

/* Arithmetic mode of vk_diffuse's fused passes.  0 (default) = bit-identical
 * with the reference's f += coef * scipy.ndimage.convolve(f, LAP, 'reflect')
 * (diffusion_field.py:385-394: summation order N, W, -4C, E, S, two roundings
 * per update, delta-then-accumulate at the end of the step).  1 = tolerance
 * mode: fma(coef, (N+S)+(E+W), (1-4coef)*C) per cell-substep (5 FP64 ops
 * instead of 6) and a final pass that writes the new field without re-reading
 * the step-start field; within ~1e-14 relative of mode 0 over a 100-substep
 * step (tests/test_stencil_modes.py).  Single-substep passes and
 * vk_diffuse_delta stay exact.  Returns the previous mode; other values only
 * query.                                                                   */
int vk_set_stencil_mode(int32_t mode);

/* out[idx] = the device's constant-rate wall clock (s_memrealtime ticks, see
 * vk_wall_clock_khz), written by one lane of a one-wave launch on `stream`.
 * Not a reference interface: the bench stamps segment boundaries inside a
 * replayed HIP graph with it (torch refuses events in graphs on ROCm).     */
int vk_timestamp(uint64_t *out, int32_t idx, vk_stream_t stream);

/* dst[0:n) = src[0:n) as the box's fastest streaming copy (one 16-B element per
 * thread, non-temporal stores): the HBM floor any stencil pass over the same
 * planes has (bench.py copy_floor).  Not a reference interface.  n even, both
 * buffers 16-B aligned.                                                     */
int vk_copy_stream(const double *src, double *dst, int64_t n, vk_stream_t stream);

/* Tick rate of vk_timestamp's clock in kHz (hipDeviceAttributeWallClockRate
 * of the current device); 0 on error.                                       */
int64_t vk_wall_clock_khz(void);

/* dst[map_row[i]*ld + a] = fields[map_field[i]*field_stride + bin_lin[a]]. */
int vk_gather(const double *fields, int64_t field_stride, const int32_t *bin_lin,
              int64_t n_agents, const int32_t *map_field, const int32_t *map_row,
              int32_t n_map, double *dst, int64_t ld, vk_stream_t stream);

/* Deterministic exchange: for each occupied bin occ_bin[b] and each map entry
 * i, field += counts[map_count[i]*ld + a] / binvol_avogadro * 1000 for its
 * agents occ_agent[occ_ptr[b]..occ_ptr[b+1]) in that (agent) order --
 * bit-identical to applying update_field_with_exchange agent by agent.   */
int vk_exchange_sorted(double *fields, int64_t field_stride, const int32_t *occ_bin,
                       const int32_t *occ_ptr, const int32_t *occ_agent, int32_t n_occ,
                       const int64_t *counts, int64_t ld, const int32_t *map_count,
                       const int32_t *map_field, int32_t n_map, double binvol_avogadro,
                       vk_stream_t stream);

/* Order-free exchange with float64 atomics (same sum, any order). */
int vk_exchange_atomic(double *fields, int64_t field_stride, const int32_t *bin_lin,
                       int64_t n_agents, const int64_t *counts, int64_t ld,
                       const int32_t *map_count, const int32_t *map_field, int32_t n_map,
                       double binvol_avogadro, vk_stream_t stream);

/* bin = floor(loc*n/bound) mod n per axis; bin_lin = (ix - row_offset)*ny + iy.
 * loc is [2][ld] (x row then y row).  ix_out (nullable) receives ix.     */
int vk_bin_sites(const double *loc, int64_t n_agents, int64_t ld, int32_t nx, int32_t ny,
                 double bound_x, double bound_y, int32_t row_offset, int32_t *bin_lin,
                 int32_t *ix_out, vk_stream_t stream);

/* ---------------------------------------------------------------------------
 * Cell growth, derivers and division
 *
 *   vk_cell_step
 *       replaces, per agent and step, GrowthProtein.next_update
 *       (vivarium/processes/growth_protein.py:88-107) or Growth.next_update
 *       (growth.py:101-107) + DivisionVolume.next_update (division_volume.py:
 *       39-45) -- all from the step-start state -- followed by the derivers
 *       TreeMass (tree_mass.py:10-18) and DeriveGlobals.next_update
 *       (derive_globals.py:131-152) on the updated state.  Writes divide[a].
 *   vk_divide_plan + vk_divide_gather / vk_divide_lineage / vk_divide_locations
 *       replace MetaDivision.next_update (meta_division.py:60-88) and the
 *       `_divide` branch of Store.apply_update (core/experiment.py:664-697)
 *       with its dividers (core/registry.py:197-280): the new agent order is
 *       the survivors in order, then daughters id+'0', id+'1' of each mother
 *       in mother order; mothers are removed.
 * ------------------------------------------------------------------------- */

/* Rows of the per-agent cell array cell[VK_CELL_ROWS][ld] ("global" port). */
enum vk_cell_row {
    VK_CELL_MASS = 0,         /* fg                                  split */
    VK_CELL_VOLUME = 1,       /* fL                                  split */
    VK_CELL_LENGTH = 2,       /* um                                  split */
    VK_CELL_SURFACE_AREA = 3, /* um^2                                split */
    VK_CELL_PROTEIN = 4,      /* counts (float, as the reference)    split */
    VK_CELL_ANGLE = 5,        /* rad (orientation for daughter locations) set */
    VK_CELL_ROWS = 6
};

enum vk_growth_model {
    VK_GROWTH_PROTEIN = 0,  /* GrowthProtein + TreeMass; divide when protein >= divide_protein */
    VK_GROWTH_MASS = 1      /* Growth (mass*factor); DivisionVolume: divide when volume >= division_volume */
};

enum vk_rng {
    VK_RNG_STREAM = 0,      /* uniforms u[a] supplied by the caller in agent order (e.g. numpy's
                               MT19937 stream, which replays the reference exactly)            */
    VK_RNG_PHILOX = 1       /* Philox4x32-10 counter = (step, root, path lo, path hi),
                               key = (seed lo + depth, seed hi): order-independent               */
};

typedef struct vk_cell_params {
    int32_t model;            /* vk_growth_model                                     */
    int32_t rng;              /* vk_rng (VK_GROWTH_PROTEIN only)                     */
    double factor;            /* exp(growth_rate * dt), evaluated by the host        */
    double divide_protein;    /* GrowthProtein: 2 * initial protein                  */
    double division_volume;   /* DivisionVolume threshold (fL)                       */
    double protein_mw;        /* g/mol                                               */
    double avogadro;          /* 1/mol                                               */
    double fg_per_g;          /* g -> fg factor as the reference's units evaluate it */
    double density;           /* g/L                                                 */
    double volume_to_fl;      /* fg*L/g -> fL factor as the reference evaluates it   */
    /* capsule constants of the (colony-wide) width w, r = w/2, evaluated by the host
       exactly as derive_globals.py:20-50 writes them                                 */
    double cap_volume;        /* (4/3)*PI*r**3                                       */
    double cap_area;          /* PI*r**2                                             */
    double two_r;             /* 2*r                                                 */
    double width;             /* w                                                   */
    double sa_const;          /* 3*PI*r**2                                           */
    double sa_lin;            /* 2*PI*r                                              */
    uint64_t seed;            /* VK_RNG_PHILOX                                       */
    uint64_t step;            /* VK_RNG_PHILOX counter word                          */
} vk_cell_params;

/* Lineage (phylogeny id) of agent a: root[a] indexes the caller's root ids,
 * the id string is root id + the depth[a] low bits of path[a], MSB first.   */

/* Growth process + derivers for agents [0, n).  u: [ld] uniforms (VK_RNG_STREAM)
 * or NULL; root/depth/path: lineage (VK_RNG_PHILOX) or NULL.  cell rows and
 * mmol_to_counts are updated in place; divide[a] = 0/1.                     */
int vk_cell_step(const vk_cell_params *p, int64_t n_agents, int64_t ld, double *cell,
                 double *mmol_to_counts, const double *u, const int32_t *root,
                 const int32_t *depth, const uint64_t *path, int32_t *divide,
                 vk_stream_t stream);

/* Division plan: src_index[j] = source agent of new slot j, kind[j] = -1 for a
 * survivor, 0 / 1 for daughter 0 / 1 (j < n_agents + n_divide).  n_out: one
 * device int64 (new agent count).  scratch: >= vk_divide_scratch_bytes(n).
 * The new count must fit the destination capacity the caller then uses.    */
int64_t vk_divide_scratch_bytes(int64_t n_agents);
int vk_divide_plan(const int32_t *divide, int64_t n_agents, int32_t *src_index, int32_t *kind,
                   int64_t *n_out, void *scratch, vk_stream_t stream);

enum vk_divider {
    VK_DIVIDE_SET = 0,     /* both daughters copy the mother's value (no divider)  */
    VK_DIVIDE_SPLIT = 1,   /* float64 halves (registry.py divide_split, floats)     */
    VK_DIVIDE_ZERO = 2     /* daughters get 0 (divide flags: meta_division.py:21)   */
};

/* dst[r*ld_dst + j] = divider(src[r*ld_src + src_index[j]]) for rows [0, rows),
 * slots [0, n_out); elem_bytes 4 or 8 (SPLIT: 8 = float64 only).            */
int vk_divide_gather(int64_t n_out, const int32_t *src_index, const int32_t *kind,
                     const void *src, int64_t ld_src, void *dst, int64_t ld_dst, int32_t rows,
                     int32_t elem_bytes, int32_t divider, vk_stream_t stream);

/* Lineage divider (daughter_phylogeny_id, meta_division.py:15-18): daughter k
 * of (root, depth, path) is (root, depth+1, path*2+k).  Sets *overflow (device
 * int32, nullable) when a lineage would exceed 64 generations.              */
int vk_divide_lineage(int64_t n_out, const int32_t *src_index, const int32_t *kind,
                      const int32_t *root_src, const int32_t *depth_src, const uint64_t *path_src,
                      int32_t *root_dst, int32_t *depth_dst, uint64_t *path_dst,
                      int32_t *overflow, vk_stream_t stream);

/* daughter_locations (multibody_physics.py:77-87): daughter k of a mother at
 * (x, y) with length L and angle t sits at (x + L*q*cos t, y + L*q*sin t),
 * q = -0.25 / +0.25.  loc_* are [2][ld] (x row, y row); the mother's length
 * and angle are read from the gathered cell rows (length already split).    */
int vk_divide_locations(int64_t n_out, const int32_t *src_index, const int32_t *kind,
                        const double *loc_src, int64_t ld_src, double *loc_dst, int64_t ld_dst,
                        const double *cell_dst, vk_stream_t stream);

/* ---------------------------------------------------------------------------
 * Kremling 2007 sugar transport: the reference's only odeint
 * call, Transport.next_update (vivarium/processes/Kremling2007_transport.py:
 * 218-427).  DEFAULT_PARAMETERS (:19-70) in this field order; units as the
 * reference (time in hours).
 * ------------------------------------------------------------------------- */
typedef struct vk_kremling_params {
    double k1, k2, k3, K1, K2, K3, kd, m, n, x0, kg6p, Kg6p, kptsup, Kglc, Keiiap, klac, Km_lac,
        Kieiia, kgly, kpyk, kpdh, kpts, km_pts, mw1, mw2, mw3, Y1_sim, Y2_sim, Y3_sim, K, kb, ksyn,
        KI;
} vk_kremling_params;

/* state[15][ld]: mass, UHPT, LACZ, PTSG, G6P, PEP, PYR, XP, GLC[e], G6P[e],
 * LCTS[e], then 4 scratch rows (flux integrals GLCpts, PPS, PYK, glc__D_e).
 * Integrates over the reference's grid t_i = i*grid_h (hours), i <
 * n_grid (np.arange(0, dt/3600, 0.01/3600): 100 points, last at 0.99 s),
 * landing on every grid point.  Rows 0-7 := y(t_last); rows 8-10 (external)
 * are left as they were; flux[4][ld] := mean over the grid points of the
 * integrals; counts[3][ld] := int(N_A * V * ((c(t_last) - c(0)) * 1e-3)) for
 * GLC, G6P, LCTS (flux_conversion.millimolar_to_counts), V = volume_fl*1e-15.
 * h_state (nullable, in/out, hours): step-size carry-over.                  */
int vk_kremling_step(const vk_kremling_params *params, int64_t n_agents, int64_t ld,
                     double timestep_h, double grid_h, int32_t n_grid, double rtol, double atol,
                     int32_t max_steps, double *state, const double *volume_fl, double avogadro,
                     double *h_state, double *flux, int64_t *counts, int32_t *status,
                     int32_t *nsteps, vk_stream_t stream);

/* ---------------------------------------------------------------------------
 * ODE gene expression with boolean regulation:
 * ODE_expression.next_update (vivarium/processes/ode_expression.py:265-303)
 * with regulation rules (vivarium/library/regulation_logic.py) compiled by
 * lens_amd/expression.py into postfix programs.
 * ------------------------------------------------------------------------- */
enum vk_expr_op {
    VK_EXPR_CMP_GT = 0,   /* push conc[a] > thr[b]                       */
    VK_EXPR_CMP_LT = 1,   /* push conc[a] < thr[b]                       */
    VK_EXPR_PRESENT = 2,  /* push conc[a] > 0  (a lone numeric operand)  */
    VK_EXPR_CONST = 3,    /* push a != 0                                 */
    VK_EXPR_NOT = 4,
    VK_EXPR_AND = 5,
    VK_EXPR_OR = 6
};

/* All pointers are DEVICE arrays owned by the caller.  Programs are
 * [op, a, b] int32 triples; transcript t's rule is code[prog_ptr[t] ..
 * prog_ptr[t+1]) (empty = unregulated).                                     */
typedef struct vk_expr_table {
    int32_t n_tx, n_tl;
    const int32_t *tx_row;        /* [n_tx] state row of each transcript      */
    const double *tx_rate;        /* [n_tx] transcription rate                */
    const double *tx_deg;         /* [n_tx] degradation rate (0 if absent)    */
    const int32_t *tx_prog_ptr;   /* [n_tx+1]                                 */
    const int32_t *code;          /* [3 * n_instr]                            */
    const double *thr;            /* thresholds                               */
    const int32_t *tl_row;        /* [n_tl] state row of each protein         */
    const int32_t *tl_mrna_row;   /* [n_tl] its transcript's row              */
    const double *tl_rate;        /* [n_tl] translation rate                  */
    const double *tl_deg;         /* [n_tl] degradation rate                  */
    double leak_p;                /* 1 - exp(-(-log(1 - rate)) * dt), host    */
    double leak_magnitude;
} vk_expr_table;

/* update[j][ld] := the reference's {'internal': {...}} values, transcripts
 * (j < n_tx) then proteins, all from the step-start conc; accumulate != 0
 * then adds them into conc (the accumulate updater).  u[n_tx][ld] (nullable):
 * uniforms for the leak draws of inhibited transcripts (NULL: no leak).      */
int vk_expression_step(const vk_expr_table *t, int64_t n_agents, int64_t ld, double dt, double *conc,
                       double *update, const double *u, int32_t accumulate, vk_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* VK_KINETICS_H */
