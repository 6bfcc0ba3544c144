#= DiffusionMCMCToolsAMD — Julia binding of libdmt (include/dmt.h) for DiffusionMCMCTools.jl.

Loading this module next to DiffusionMCMCTools makes the reference's unchanged caller code run
on the GPU: the reference's own constructors (`SamplingPair(AuxLaw, recording, tts)`,
`SamplingEnsemble(AuxLaw, recordings, tts)`, `BiBlock(sp, …)`, `BlockCollection(sp, …)`,
`BlockEnsemble(se, …)`) build device containers, and every function the tutorials call is a
METHOD of the reference's generic function (imported from DiffusionMCMCTools, or GuidedProposals'
`GP.set_obs!`, `GP.recompute_guiding_term!`, `GP.loglikhd`, `GP.equalize_obs_params!`) on the
device types, with the reference's field accesses (`bb.b.ll`, `bb.b°.ll`, `bb.b.XX`, `sp.u.XX`,
`se.recordings`).  Each method is one `ccall` over a block range; host arrays are the
reference's own containers reinterpreted (Vector{SVector{d,Float64}} == double[npts][d]).
`use_device!(false)` restores the reference's CPU constructors.

No Julia toolchain exists in the build image, so this file is shipped as source and is not run
by the test suite; tests/test_julia_binding.py checks every `ccall` type tuple against the
prototypes of include/dmt.h and that every name the reference's tutorials call is defined here
as a method of the reference's (or GuidedProposals') generic function.  The Python mirror
(../api.py, ../functions.py) calls the same entry points and is tested end to end, including
the tutorial loops verbatim (examples/reference_tutorials.py).  See INTEGRATION.md.
=#
module DiffusionMCMCToolsAMD

using StaticArrays
using LinearAlgebra: I, det, inv

import GuidedProposals
const GP = GuidedProposals
import DiffusionDefinition
const DD = DiffusionDefinition
import DiffusionMCMCTools
import DiffusionMCMCTools: draw_proposal_path!, accept_reject_proposal_path!, loglikhd!,
    loglikhd°!, fetch_ll, fetch_ll°, save_ll!, set_ll!, set_accepted!, swap_paths!, swap_XX!,
    swap_WW!, swap_PP!, swap_ll!, ll_of_accepted, accpt_rate, recompute_path!, find_W_for_X!,
    set_proposal_law!, SamplingUnit, SamplingPair, SamplingEnsemble, Block, BiBlock,
    BlockCollection, BlockEnsemble, ParamNamesBlock, ParamNamesRecording, ParamNamesAllObs

# device-only names (everything the reference's callers use is a method of its own functions)
export DeviceSamplingEnsemble, DeviceSamplingPair, DeviceSamplingUnit, DeviceBlockEnsemble,
    DeviceBlockCollection, DeviceBiBlock, DeviceBlock, use_device!, mcmc_step!, mcmc_run!,
    download_XX, download_WW, upload_obs!, snapshot_every!, law_record, guiding_linear, sync,
    upload_aux!, upload_aux_a!, device_model, device_aux

const libdmt = get(ENV, "DMT_LIB", joinpath(@__DIR__, "..", "libdmt.so"))

# ---- constants (include/dmt.h)
const DMT_MODEL_OU, DMT_MODEL_FHN, DMT_MODEL_LORENZ = Int32(0), Int32(1), Int32(2)
const DMT_F64, DMT_F32 = Int32(0), Int32(1)
const DMT_MAP_AUTO = Int32(0)
const DMT_U, DMT_UPROP = Int32(0), Int32(1)
const DMT_LAW_PP, DMT_LAW_PPB = Int32(0), Int32(1)
const DMT_SWAP_XX, DMT_SWAP_WW, DMT_SWAP_PP, DMT_SWAP_LL = Int32(1), Int32(2), Int32(4), Int32(8)
const DMT_BLK_LL, DMT_BLK_LLPROP, DMT_BLK_LL_HIST, DMT_BLK_LLPROP_HIST, DMT_BLK_ACC_HIST =
    Int32(0), Int32(1), Int32(2), Int32(3), Int32(4)
const DMT_LAW_STRIDE = 64
# draws with no key take the handle's stream counter, as the reference's take the global RNG
# (src/biblock.jl:94-99,122); explicit salts must stay below DMT_SALT_LIMIT
const DMT_RNG_AUTO = typemax(UInt32)
const DMT_SALT_LIMIT = UInt32(0x40000000)
_key(iter, salt) = (iter === nothing && salt === nothing) ? (0, DMT_RNG_AUTO) :
    (something(iter, 0), UInt32(something(salt, 0)))

struct dmt_model
    model::Int32
    precision::Int32
    d::Int32
    m::Int32
end

struct dmt_structure
    n_recordings::Int64
    n_segments::Ptr{Int32}
    n_points::Ptr{Int32}
end

struct dmt_config
    seed::UInt64
    device::Int32
    grid_shared::Int32
    mapping::Int32
end

function check(st::Int32)
    st == 0 && return nothing
    msg = unsafe_string(ccall((:dmt_last_error, libdmt), Cstring, ()))
    error("libdmt error $st: $msg")
end

# `using DiffusionMCMCToolsAMD` sends the reference's SamplingPair / SamplingEnsemble
# constructors to the device; use_device!(false) gives the CPU ones back
const DEVICE = Ref(true)
const DEVICE_OPTS = Ref{Any}((device=0, seed=0))
use_device!(on::Bool=true; device::Integer=0, seed::Integer=0) =
    (DEVICE[] = on; DEVICE_OPTS[] = (device=device, seed=seed); on)

# ============================================================ SamplingEnsemble (device)
"""
    DeviceSamplingEnsemble(model, d, m, n_points; precision, seed, device, grid_shared)

Device containers of a `SamplingEnsemble` (src/sampling_ensemble.jl:13-41): XX/WW of `u` and
`u°` for every recording.  `n_points[r][k]` = grid points of segment k of recording r.
"""
mutable struct DeviceSamplingEnsemble
    h::Ptr{Cvoid}
    model::Int32
    d::Int
    m::Int
    n_points::Vector{Vector{Int}}
    P::Int
    t::Vector{Float64}       # host copy of the time grids (trajectory views)
    function DeviceSamplingEnsemble(model::Integer, d::Integer, m::Integer, n_points;
                                    precision=DMT_F64, seed::Integer=0, device::Integer=0,
                                    grid_shared::Bool=false, mapping=DMT_MAP_AUTO)
        nseg = Int32[length(r) for r in n_points]
        npts = Int32[n for r in n_points for n in r]
        h = Ref{Ptr{Cvoid}}(C_NULL)
        mdl = Ref(dmt_model(model, precision, d, m))
        GC.@preserve nseg npts begin
            st = Ref(dmt_structure(length(nseg), pointer(nseg), pointer(npts)))
            cfg = Ref(dmt_config(UInt64(seed), device, grid_shared, mapping))
            check(ccall((:dmt_create, libdmt), Int32,
                        (Ref{Ptr{Cvoid}}, Ref{dmt_model}, Ref{dmt_structure}, Ref{dmt_config}),
                        h, mdl, st, cfg))
        end
        se = new(h[], Int32(model), d, m, [collect(Int, r) for r in n_points], sum(npts),
                 Float64[])
        finalizer(se) do x
            x.h == C_NULL || ccall((:dmt_destroy, libdmt), Int32, (Ptr{Cvoid},), x.h)
            x.h = C_NULL
        end
        se
    end
end

"""
    sync(x)

Wait for the ensemble's queued device work and stop a resident service launch (include/dmt.h,
"Resident service"): call it before a device-wide synchronisation issued outside libdmt.
"""
sync(se::DeviceSamplingEnsemble) = check(ccall((:dmt_sync, libdmt), Int32, (Ptr{Cvoid},), se.h))

"Concatenate per-segment trajectories (Vector{SVector}) recording-major into one flat buffer."
flatten_paths(segs) = reduce(vcat, (collect(reinterpret(Float64, s)) for s in segs))

function upload_grid!(se::DeviceSamplingEnsemble, t::Vector{Float64})
    check(ccall((:dmt_upload_grid, libdmt), Int32, (Ptr{Cvoid}, Ptr{Float64}), se.h, t))
    se.t = copy(t)
    nothing
end

"""
    upload_law!(se, unit, kind, H, F, laws; H_shared=false)

Guiding-term tables of `u.PP`/`u°.PP` (kind `DMT_LAW_PP`) or `PPb` (`DMT_LAW_PPB`): packed
`H` (upper triangle, row-major, per grid point), `F`, and one law record per segment
(`DMT_LAW_STRIDE` doubles, layout in include/dmt.h).  Pass `nothing` to keep a table.
"""
function upload_law!(se::DeviceSamplingEnsemble, unit, kind, H, F, laws; H_shared=false)
    p(x) = x === nothing ? Ptr{Float64}(C_NULL) : pointer(x)
    GC.@preserve H F laws check(ccall((:dmt_upload_law, libdmt), Int32,
        (Ptr{Cvoid}, Int32, Int32, Ptr{Float64}, Int32, Ptr{Float64}, Ptr{Float64}),
        se.h, unit, kind, p(H), H_shared, p(F), p(laws)))
end

"init_paths!-style upload: X (and W, cumulative) of a unit, flat reference layout."
function set_paths!(se::DeviceSamplingEnsemble, unit, X, W=nothing)
    p(x) = x === nothing ? Ptr{Float64}(C_NULL) : pointer(x)
    GC.@preserve X W check(ccall((:dmt_set_paths, libdmt), Int32,
        (Ptr{Cvoid}, Int32, Ptr{Float64}, Ptr{Float64}), se.h, unit, p(X), p(W)))
end

function _download(se::DeviceSamplingEnsemble, unit, what, C)
    out = Vector{Float64}(undef, se.P * C)
    check(ccall((:dmt_download_paths, libdmt), Int32, (Ptr{Cvoid}, Int32, Int32, Ptr{Float64}),
                se.h, unit, what, out))
    collect(reinterpret(SVector{C,Float64}, out))
end
download_XX(se::DeviceSamplingEnsemble, unit=DMT_U) = _download(se, unit, 0, se.d)
download_WW(se::DeviceSamplingEnsemble, unit=DMT_U) = _download(se, unit, 1, se.m)

# flat point offsets of the segments, recording-major
_pt_off(se::DeviceSamplingEnsemble) = cumsum([0; [n for r in se.n_points for n in r]])
_seg0(se::DeviceSamplingEnsemble, r) = sum(length.(se.n_points[1:r-1]); init=0)

"Per-segment trajectories (t, x) of segments `segs` (1-based, global) from a flat download."
function _trajectories(se::DeviceSamplingEnsemble, A, segs)
    off = _pt_off(se)
    map(segs) do g
        rows = off[g]+1:off[g+1]
        # DiffusionDefinition's trajectory(t, x): the type sp.u.XX holds in the reference
        DD.trajectory(se.t[rows], A[rows])
    end
end

# ---- path snapshots: `append!(paths, [deepcopy(bb.b.XX)])` (docs/src/tutorials/biblock/
# smoothing.md:55) without leaving the GPU; slots are 0-based, what_mask 1 = XX, 2 = WW, 3 = both
reserve_snapshots!(se::DeviceSamplingEnsemble, n_slots; what_mask=1) =
    check(ccall((:dmt_snapshot_reserve, libdmt), Int32, (Ptr{Cvoid}, Int32, Int64),
                se.h, what_mask, n_slots))
snapshot!(se::DeviceSamplingEnsemble, slot, mcmciter; unit=DMT_U) =
    check(ccall((:dmt_snapshot_take, libdmt), Int32, (Ptr{Cvoid}, Int32, Int64, Int64),
                se.h, unit, slot, mcmciter))
function snapshot(se::DeviceSamplingEnsemble, slot; what=0)
    C = what == 0 ? se.d : se.m
    out = Vector{Float64}(undef, se.P * C)
    it = Ref{Int64}(0)
    check(ccall((:dmt_snapshot_download, libdmt), Int32,
                (Ptr{Cvoid}, Int32, Int64, Ptr{Float64}, Ref{Int64}), se.h, what, slot, out, it))
    collect(reinterpret(SVector{C,Float64}, out)), it[]
end
# snapshots inside mcmc_run!: u after every iteration k with k % every == 0 → slots slot0, …
# (a ring), no host round trip; every = 0 turns it off
snapshot_every!(se::DeviceSamplingEnsemble, every; slot0=0) =
    check(ccall((:dmt_set_run_snapshots, libdmt), Int32, (Ptr{Cvoid}, Int64, Int64),
                se.h, every, slot0))
write_snapshots(se::DeviceSamplingEnsemble, path::AbstractString, s0, s1) =
    check(ccall((:dmt_snapshot_write, libdmt), Int32, (Ptr{Cvoid}, Cstring, Int64, Int64),
                se.h, path, s0, s1))

"draw_proposal_path!(u::SamplingUnit) for recordings r0+1:r1 (src/sampling_unit.jl:118)."
function draw_unit!(se::DeviceSamplingEnsemble, unit, r0, r1; Z=nothing, iter=nothing,
                    salt=nothing)
    iter, salt = _key(iter, salt)
    ll = Vector{Float64}(undef, r1 - r0)
    ok = Vector{UInt8}(undef, r1 - r0)
    pz = Z === nothing ? Ptr{Float64}(C_NULL) : pointer(Z)
    GC.@preserve Z check(ccall((:dmt_draw_unit, libdmt), Int32,
        (Ptr{Cvoid}, Int32, Int64, Int64, Ptr{Float64}, Int64, UInt32, Ptr{Float64}, Ptr{UInt8}),
        se.h, unit, r0, r1, pz, iter, salt, ll, ok))
    Bool.(ok), ll
end

# ============================================================ containers from laws
# The reference builds its containers from laws: SamplingUnit(aux_laws, recording, tts;
# aux_laws_blocking, artificial_noise) → build_guid_prop / guid_prop_for_blocking
# (src/sampling_unit.jl:55-74).  The functions below do the same for the device from the
# laws' coefficients — the target's parameters and σ, each auxiliary law's (B̃, β̃, σ̃) — with
# the exact backward filter of dmt_guiding_linear (the Python mirror
# `SamplingEnsemble.from_recordings`, tests/test_api.py, is the tested twin).

"Upper triangle of a symmetric matrix, row-major (the device's packed H)."
packed(M::AbstractMatrix) = [M[i, j] for i in 1:size(M, 1) for j in i:size(M, 2)]
unpacked(p::AbstractVector, d) = (M = zeros(d, d); k = 0;
    for i in 1:d, j in i:d; k += 1; M[i, j] = M[j, i] = p[k]; end; M)

"""
    law_record(θrec, σ, B̃, β̃, σ̃, c0; anchor=nothing, time_dependent=false)

One segment's law record (DMT_LAW_STRIDE doubles, include/dmt.h): θrec = the target's
parameters in the device order (OU: Θ row-major at 1:d², μ at 10:9+d; FHN: 1/ϵ, s, γ, β, ϵ, σ;
Lorenz: s, r, β), σ (d×m), the auxiliary law's B̃, β̃, σ̃, c(t₀), and the linearisation point
of a linearised auxiliary law (FitzHughNagumoAux: y_T; Lorenz: x_T).  `time_dependent=true`:
B̃(t), β̃(t) vary within the segment and come from `upload_aux!` (B̃, β̃ here: any one value).
"""
function law_record(θrec, σ::AbstractMatrix, B̃::AbstractMatrix, β̃, σ̃::AbstractMatrix, c0;
                    anchor=nothing, time_dependent=false)
    d, m = size(σ)
    hp = d * (d + 1) ÷ 2
    rec = zeros(DMT_LAW_STRIDE)
    rec[1:length(θrec)] .= θrec                                    # DMT_LAW_THETA 0
    rec[17:16+d*m] .= vec(permutedims(σ))                          # DMT_LAW_SIGMA 16
    a, ã = σ * σ', σ̃ * σ̃'
    rec[26:25+hp] .= packed(a)                                      # DMT_LAW_A 25
    rec[32:31+d*d] .= vec(permutedims(B̃))                          # DMT_LAW_BT 31
    rec[41:40+d] .= β̃                                              # DMT_LAW_BETA 40
    da = a - ã
    rec[44:43+hp] .= packed(da)                                     # DMT_LAW_DA 43
    rec[50] = c0                                                    # DMT_LAW_C0 49
    rec[51] = any(!iszero, da) ? 1.0 : 0.0                          # DMT_LAW_TRACE 50
    d == m && (rec[52:51+d*d] .= vec(permutedims(inv(σ))))          # DMT_LAW_SIGINV 51
    if anchor !== nothing                                           # DMT_LAW_ANCHOR 60
        rec[61:60+length(anchor)] .= anchor
        rec[64] = 1.0                                               # DMT_LAW_AUXLIN 63
    end
    time_dependent && (rec[16] = 1.0)                               # DMT_LAW_AUXTD 15
    rec
end

"""
    upload_aux!(se, kind, aux)

Time-dependent auxiliary laws (dmt_upload_aux): `aux` is (d² + d) × P — column i holds
B̃(t_i) (row-major) then β̃(t_i) at grid point i of every segment — for the laws of `kind`
(0: PP, 1: PPb) of u and u°; `nothing` removes it.  Used by the segments whose law record has
`time_dependent=true`.  Non-linear drifts only.
"""
function upload_aux!(se::DeviceSamplingEnsemble, kind, aux)
    p(x) = x === nothing ? Ptr{Float64}(C_NULL) : pointer(x)
    GC.@preserve aux check(ccall((:dmt_upload_aux, libdmt), Int32,
        (Ptr{Cvoid}, Int32, Ptr{Float64}), se.h, kind, p(aux)))
end

"""
    upload_aux_a!(se, kind, aux, ncols)

dmt_upload_aux_a: `aux` is ncols × P with ncols = d² + d (as `upload_aux!`) or d² + d + d(d+1)/2
— B̃(t_i), β̃(t_i) and ã(t_i) packed — for segments whose record has DMT_LAW_AUXTD = 2 (ã(t) from
the table) or 1 (the record's ã).
"""
function upload_aux_a!(se::DeviceSamplingEnsemble, kind, aux, ncols::Integer)
    GC.@preserve aux check(ccall((:dmt_upload_aux_a, libdmt), Int32,
        (Ptr{Cvoid}, Int32, Ptr{Float64}, Int32), se.h, kind, pointer(aux), ncols))
end

"""
    guiding_linear(B̃, β̃, σ̃, t, HT, FT, cT) -> (H, F, c)

The guiding term of a linear auxiliary law on grid `t` from the end information (HT, FT, cT):
dmt_guiding_linear (the exact discrete filter, DESIGN.md §3).  H: npts × d(d+1)/2 (packed,
one row per point), F: npts × d, c: npts.
"""
function guiding_linear(B̃, β̃, σ̃, t::Vector{Float64}, HT::AbstractMatrix, FT, cT)
    d, n = length(β̃), length(t)
    hp = d * (d + 1) ÷ 2
    Bt, β, at = vec(permutedims(Float64.(B̃))), Float64.(collect(β̃)), packed(σ̃ * σ̃')
    HTp, FTv = packed(HT), Float64.(collect(FT))
    H, F, c = Matrix{Float64}(undef, hp, n), Matrix{Float64}(undef, d, n), Vector{Float64}(undef, n)
    check(ccall((:dmt_guiding_linear, libdmt), Int32,
        (Int32, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Int32, Ptr{Float64}, Ptr{Float64},
         Ptr{Float64}, Float64, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}),
        d, Bt, β, at, n, t, HTp, FTv, cT, H, F, c))
    permutedims(H), permutedims(F), c
end

"""
    guiding_linear(B̃::Function, β̃::Function, σ̃, t, HT, FT, cT) -> (H, F, c)

The guiding term of a time-dependent linear auxiliary law dX = (B̃(t)X + β̃(t))dt + σ̃dW:
dmt_guiding_linear_td, each step's exact transition taking B̃, β̃ at its left point.
"""
function guiding_linear(B̃::Function, β̃::Function, σ̃, t::Vector{Float64}, HT::AbstractMatrix, FT, cT)
    d, n = length(β̃(t[1])), length(t)
    hp = d * (d + 1) ÷ 2
    aux = Matrix{Float64}(undef, d * d + d, n)
    for i in 1:n
        aux[1:d*d, i] .= vec(permutedims(Float64.(B̃(t[i]))))
        aux[d*d+1:end, i] .= Float64.(collect(β̃(t[i])))
    end
    at, HTp, FTv = packed(σ̃ * σ̃'), packed(HT), Float64.(collect(FT))
    H, F, c = Matrix{Float64}(undef, hp, n), Matrix{Float64}(undef, d, n), Vector{Float64}(undef, n)
    check(ccall((:dmt_guiding_linear_td, libdmt), Int32,
        (Int32, Ptr{Float64}, Ptr{Float64}, Int32, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
         Float64, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}),
        d, aux, at, n, t, HTp, FTv, cT, H, F, c))
    permutedims(H), permutedims(F), c
end

"Information (H, F, c) of an observation v ~ N(L x, Σ) (ObservationSchemes LinearGsnObs)."
function obs_info(v, L::AbstractMatrix, Σ::AbstractMatrix)
    Si = inv(Σ)
    H, F = L' * Si * L, L' * Si * v
    H, F, 0.5 * v' * Si * v + 0.5 * length(v) * log(2π) + 0.5 * log(det(Σ))
end

"""
    DeviceSamplingEnsemble(model, θrec, σ, recordings, tts, aux; aux_blocking=aux,
                           artificial_noise=1e-11, blocking=true, kw...)

`SamplingEnsemble(aux_laws, recordings, tts; aux_laws_blocking, artificial_noise)` on the device
(src/sampling_ensemble.jl:20-40 → src/sampling_unit.jl:55-66): `recordings[r] = (obs = [(t, v,
L, Σ), …], x0 = …)`, `tts[r][k]` the grid of segment k, `aux(r, k, obs) -> (B̃, β̃, σ̃, anchor)`
the auxiliary law of segment k (build_guid_prop), `aux_blocking` the same for the blocking laws
(guid_prop_for_blocking).  B̃ and β̃ may be functions of t (a time-dependent linear law: the
segment's law record is flagged and its per-point table goes up with `upload_aux!`), and so may
σ̃ (then ã(t) = σ̃σ̃ᵀ(t) is tabled too: `upload_aux_a!`).  `θrec` is one law-parameter vector for
all recordings or a function `r -> θrec` (each recording's own target law).  Guiding terms
through each recording's segments, blocking laws with an exact full-state artificial end
observation (a placeholder until set_obs!), the observations for the device's re-derivations,
then init_paths! from x0.  The Python twin is `SamplingEnsemble.from_recordings` (api.py).
"""
function DeviceSamplingEnsemble(model::Integer, θrec, σ::AbstractMatrix, recordings, tts, aux;
                                aux_blocking=aux, artificial_noise=1e-11, blocking=true, kw...)
    d, m = size(σ)
    θof = θrec isa Function ? θrec : (r -> θrec)
    t_all, H_all, F_all, laws, infos = Float64[], Matrix{Float64}[], Matrix{Float64}[], Vector{Float64}[], Any[]
    Hb_all, Fb_all, lawsb = Matrix{Float64}[], Matrix{Float64}[], Vector{Float64}[]
    tab_pp, tab_b = Matrix{Float64}[], Matrix{Float64}[]   # per-point aux tables (na × npts)
    any_td, any_tda = false, false
    n_points = Vector{Int}[]
    for (r, rec) in enumerate(recordings)
        K = length(rec.obs)
        auxes = [aux(r, k, rec.obs[k]) for k in 1:K]
        info = [obs_info(o.v, o.L, o.Σ) for o in rec.obs]
        chain = Vector{Any}(undef, K)
        nxt = nothing
        for k in K:-1:1                      # segment k ends in obs k, then segment k+1 starts
            HT, FT, cT = info[k]
            if nxt !== nothing
                HT, FT, cT = HT + unpacked(nxt[1], d), FT + nxt[2], cT + nxt[3]
            end
            chain[k] = _guiding(auxes[k], Float64.(tts[r][k]), HT, FT, cT)
            nxt = (chain[k][1][1, :], chain[k][2][1, :], chain[k][3][1])
        end
        for k in 1:K
            g = Float64.(tts[r][k])
            append!(t_all, tts[r][k]); push!(H_all, chain[k][1]); push!(F_all, chain[k][2])
            push!(laws, _law_record(θof(r), σ, auxes[k], chain[k][3][1]))
            push!(tab_pp, aux_table(auxes[k], g, d))
            any_td |= is_time_dependent(auxes[k]); any_tda |= is_time_dependent_a(auxes[k])
            push!(infos, info[k])
            if blocking
                ab = aux_blocking(r, k, rec.obs[k])
                v = zeros(d); vo = collect(rec.obs[k].v); v[1:min(d, length(vo))] .= vo[1:min(d, length(vo))]
                Ha, Fa, ca = obs_info(v, Matrix(1.0I, d, d), artificial_noise * Matrix(1.0I, d, d))
                Ho, Fo, co = info[k]
                H, F, c = _guiding(ab, g, Ha + Ho, Fa + Fo, ca + co)
                push!(Hb_all, H); push!(Fb_all, F)
                push!(lawsb, _law_record(θof(r), σ, ab, c[1]))
                push!(tab_b, aux_table(ab, g, d))
                any_td |= is_time_dependent(ab); any_tda |= is_time_dependent_a(ab)
            end
        end
        push!(n_points, [length(g) for g in tts[r]])
    end
    se = DeviceSamplingEnsemble(model, d, m, n_points; kw...)
    upload_grid!(se, t_all)
    flat(Ms) = vec(permutedims(reduce(vcat, Ms)))     # point-major, components contiguous
    upload_law!(se, DMT_U, DMT_LAW_PP, flat(H_all), flat(F_all), reduce(vcat, laws))
    blocking && upload_law!(se, DMT_U, DMT_LAW_PPB, flat(Hb_all), flat(Fb_all), reduce(vcat, lawsb))
    if any_td   # per-point tables of both kinds (zero rows on time-homogeneous segments, unused)
        nc = any_tda ? d * d + d + d * (d + 1) ÷ 2 : d * d + d
        upload_aux_a!(se, DMT_LAW_PP, vec(reduce(hcat, tab_pp)[1:nc, :]), nc)
        blocking && upload_aux_a!(se, DMT_LAW_PPB, vec(reduce(hcat, tab_b)[1:nc, :]), nc)
    end
    upload_obs!(se, reduce(vcat, [packed(i[1]) for i in infos]),
                reduce(vcat, [collect(i[2]) for i in infos]), Float64[i[3] for i in infos];
                artificial_noise=artificial_noise)
    X = zeros(d, se.P)                                # init_paths!: start points, fresh draws
    p = 1
    for (r, rec) in enumerate(recordings)
        X[:, p] .= rec.x0
        p += sum(n_points[r])
    end
    set_paths!(se, DMT_U, vec(X))
    ok, _ = draw_unit!(se, DMT_U, 0, length(recordings))
    all(ok) || error("init_paths!: a recording's first draw failed")
    flat_paths(A) = collect(reinterpret(Float64, A))
    set_paths!(se, DMT_UPROP, flat_paths(download_XX(se)), flat_paths(download_WW(se)))
    se
end

# ---- auxiliary laws: (B̃, β̃, σ̃, anchor); B̃, β̃ (and σ̃) may be functions of t
is_time_dependent(a) = a[1] isa Function || a[2] isa Function || a[3] isa Function
is_time_dependent_a(a) = a[3] isa Function
_at(σ̃, t) = (S = σ̃ isa Function ? Matrix{Float64}(σ̃(t)) : Matrix{Float64}(σ̃); S * S')
_val(f, t) = f isa Function ? f(t) : f

"Guiding term (H, F, c) of auxiliary law `a` on grid `g` from the end information."
function _guiding(a, g, HT, FT, cT)
    B̃, β̃, σ̃, _ = a
    d = size(HT, 1)
    if is_time_dependent_a(a)
        tab = aux_table(a, g, d)
        hp = d * (d + 1) ÷ 2
        H, F, c = Matrix{Float64}(undef, hp, length(g)), Matrix{Float64}(undef, d, length(g)),
                  Vector{Float64}(undef, length(g))
        check(ccall((:dmt_guiding_linear_tda, libdmt), Int32,
            (Int32, Ptr{Float64}, Int32, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Float64,
             Ptr{Float64}, Ptr{Float64}, Ptr{Float64}),
            d, tab, length(g), g, packed(HT), Float64.(collect(FT)), cT, H, F, c))
        return permutedims(H), permutedims(F), c
    elseif is_time_dependent(a)
        return guiding_linear(t -> _val(B̃, t), t -> _val(β̃, t), σ̃, g, HT, FT, cT)
    end
    guiding_linear(B̃, β̃, σ̃, g, HT, FT, cT)
end

"""
    aux_table(a, g, d) -> Matrix (d² + d + d(d+1)/2) × length(g)

Per-point rows of a time-dependent auxiliary law on grid `g` (dmt_upload_aux_a layout: B̃(t_i)
row-major, β̃(t_i), ã(t_i) packed); zeros for a time-homogeneous law (its rows are unused).
"""
function aux_table(a, g, d)
    hp = d * (d + 1) ÷ 2
    T = zeros(d * d + d + hp, length(g))
    is_time_dependent(a) || return T
    B̃, β̃, σ̃, _ = a
    for (i, t) in enumerate(g)
        T[1:d*d, i] .= vec(permutedims(Float64.(_val(B̃, t))))
        T[d*d+1:d*d+d, i] .= Float64.(collect(_val(β̃, t)))
        T[d*d+d+1:end, i] .= packed(_at(σ̃, t))
    end
    T
end

"Law record of a segment with auxiliary law `a` (time-dependent laws flagged, DMT_LAW_AUXTD)."
function _law_record(θrec, σ, a, c0)
    B̃, β̃, σ̃, an = a
    d = size(σ, 1)
    if is_time_dependent(a)
        rec = law_record(θrec, σ, zeros(d, d), zeros(d), σ̃ isa Function ? σ : σ̃, c0;
                         time_dependent=true)
        is_time_dependent_a(a) && (rec[16] = 2.0)   # DMT_LAW_AUXTD = 2: ã(t) from the table
        return rec
    end
    law_record(θrec, σ, B̃, β̃, σ̃, c0; anchor=an)
end

# ---- the reference's (aux_laws, recording(s), tts) constructors on the device
# The target law of a recording is `recording.P` (ObservationSchemes recordings are
# (P, obs, t0, x0_prior), docs/src/get_started/overview.md:18-20); its observations are
# LinearGsnObs with fields t, obs, L, Σ (docs/src/tutorials/preamble.md:80-86).  Models are
# recognised by their DiffusionDefinition names or fields; extend `device_model` for others.
# Every DMT_MODEL_* of include/dmt.h has a branch (tests/test_julia_binding.py checks it).
"""
    device_model(P) -> (kind, θrec, σ)

The device model of a DiffusionDefinition target law:
* DMT_MODEL_OU — an Ornstein–Uhlenbeck law dX = −Θ(X − μ)dt + σdW: DiffusionDefinition's
  `OrnsteinUhlenbeck(θ, μ, σ)` (scalar, d = 1) or any law with fields `Θ` (or `θ`), `μ`, `σ`
  (d ≤ 3; matrices, vectors or scalars) — the north star's 2-D OU bridge;
* DMT_MODEL_FHN — FitzHughNagumo (θ = ϵ, s, γ, β, σ — positional, `FitzHughNagumo(θ...)` at
  docs/src/tutorials/preamble.md:78);
* DMT_MODEL_LORENZ — Lorenz / Lorenz63 (s, r, β[, σ₁, σ₂, σ₃]).
"""
function device_model(P)
    name = nameof(typeof(P))
    if name === :FitzHughNagumo
        ϵ, s, γ, β, σ = (getfield(P, i) for i in 1:5)
        return DMT_MODEL_FHN, [1 / ϵ, s, γ, β, ϵ, σ], reshape([0.0, σ], 2, 1)
    elseif name === :Lorenz || name === :Lorenz63
        s, r, β = (getfield(P, i) for i in 1:3)
        σ = nfields(P) >= 6 ? [getfield(P, 4), getfield(P, 5), getfield(P, 6)] : [1.0, 1.0, 1.0]
        return DMT_MODEL_LORENZ, [s, r, β], Matrix{Float64}(LinearAlgebra_diag(σ))
    elseif name === :OrnsteinUhlenbeck || name === :OU || name === :OrnsteinUhlenbeck2D ||
           (hasproperty(P, :μ) && hasproperty(P, :σ) && (hasproperty(P, :Θ) || hasproperty(P, :θ)))
        Θ = hasproperty(P, :Θ) ? getproperty(P, :Θ) :
            hasproperty(P, :θ) ? getproperty(P, :θ) : getfield(P, 1)
        μ = hasproperty(P, :μ) ? getproperty(P, :μ) : getfield(P, 2)
        σ = hasproperty(P, :σ) ? getproperty(P, :σ) : getfield(P, 3)
        μv = μ isa Number ? [Float64(μ)] : Float64.(collect(μ))
        d = length(μv)
        Θm = Θ isa Number ? Float64(Θ) * Matrix(1.0I, d, d) : Matrix{Float64}(reshape(collect(Θ), d, d))
        σm = σ isa Number ? Float64(σ) * Matrix(1.0I, d, d) :
             σ isa AbstractVector ? Matrix{Float64}(LinearAlgebra_diag(Float64.(σ))) : Matrix{Float64}(σ)
        d <= 3 || error("DiffusionMCMCToolsAMD: OU of dimension $d (the device holds d ≤ 3)")
        θrec = zeros(12)
        θrec[1:d*d] .= vec(permutedims(Θm))            # Θ row-major (DMT_LAW_THETA 0)
        θrec[10:9+d] .= μv                               # μ at 9
        return DMT_MODEL_OU, θrec, σm
    end
    error("DiffusionMCMCToolsAMD: no device model for $(name); extend device_model")
end
LinearAlgebra_diag(v) = [i == j ? v[i] : 0.0 for i in 1:length(v), j in 1:length(v)]

"""
    device_aux(kind, θrec, σ, o) -> (B̃, β̃, σ̃, anchor)

The auxiliary law of a segment ending in observation `o` that an auxiliary-law TYPE stands for
(the tutorials pass `FitzHughNagumoAux`): the target linearised at the observed value
(FitzHughNagumoAux; the Lorenz aux of config C5) or, for a linear target (OU), the target law
itself (B̃ = −Θ, β̃ = Θμ, σ̃ = σ: the guided proposal is then exact).  In the arithmetic order of
the device's re-derivation in set_proposal_law! and of the Python twin (models.py), so host and
device laws agree bit for bit.
"""
function device_aux(kind, θrec, σ, o)
    if kind == DMT_MODEL_FHN
        e, s, γ, β = θrec[5], θrec[2], θrec[3], θrec[4]
        y = Float64(o.v[1])
        B̃ = [(1.0 - 3.0 * (y * y)) / e  -1.0 / e; γ  -1.0]
        β̃ = [(s + 2.0 * (y * y * y)) / e, β]
        return B̃, β̃, σ, [y]
    elseif kind == DMT_MODEL_OU
        d = size(σ, 1)
        Θ = permutedims(reshape(θrec[1:d*d], d, d))
        μ = θrec[10:9+d]
        β̃ = [sum(Θ[i, j] * μ[j] for j in 1:d) for i in 1:d]   # left to right, no fma
        return -Θ, β̃, σ, nothing
    else
        s, r, b = θrec[1], θrec[2], θrec[3]
        x0, x1, x2 = Float64.(o.v[1:3])
        J = [-s s 0.0; r-x2 -1.0 -x0; x1 x0 -b]
        f = [s * (x1 - x0), x0 * (r - x2) - x1, x0 * x1 - b * x2]
        β̃ = [f[i] - ((J[i, 1] * x0 + J[i, 2] * x1) + J[i, 3] * x2) for i in 1:3]
        return J, β̃, σ, [x0, x1, x2]
    end
end

_obs(o) = (t = o.t, v = collect(Float64, o.obs), L = Matrix{Float64}(o.L), Σ = Matrix{Float64}(o.Σ))

"""
    _as_aux(a, σ) -> (B̃, β̃, σ̃, anchor)

One auxiliary law given by the caller: a tuple (B̃, β̃[, σ̃[, anchor]]) or a NamedTuple with
fields B̃ (or B), β̃ (or β), optionally σ̃ (or σ) and anchor — B̃, β̃, σ̃ constants or functions of
t (a time-dependent linear law, GuidedProposals' `aux_laws` varying in t).  σ̃ defaults to the
target's σ.
"""
function _as_aux(a, σ)
    if a isa NamedTuple
        B̃ = haskey(a, :B̃) ? a.B̃ : a.B
        β̃ = haskey(a, :β̃) ? a.β̃ : a.β
        σ̃ = haskey(a, :σ̃) ? a.σ̃ : haskey(a, :σ) ? a.σ : σ
        return B̃, β̃, σ̃, get(a, :anchor, nothing)
    end
    length(a) >= 2 || error("an auxiliary law is (B̃, β̃[, σ̃[, anchor]])")
    (a[1], a[2], length(a) >= 3 ? a[3] : σ, length(a) >= 4 ? a[4] : nothing)
end

"""
    aux_function(aux_laws, kind, θof, σ, Ps) -> (r, k, o) -> (B̃, β̃, σ̃, anchor)

The reference's `aux_laws` argument (src/sampling_unit.jl:55-60), as the Python twin
`api._aux_callable` reads it: `nothing` or an auxiliary-law TYPE (`FitzHughNagumoAux`) — the
law `device_aux` derives for the target at the segment's observation; a function
`(P, obs) -> law` of recording r's target `Ps[r]`; one law (tuple / NamedTuple, `_as_aux`) for
every segment; or a vector of those per segment k.
"""
function aux_function(aux_laws, kind, θof, σ, Ps)
    (aux_laws === nothing || aux_laws isa Type) &&
        return (r, k, o) -> device_aux(kind, θof(r), σ, o)
    if aux_laws isa AbstractVector
        return function (r, k, o)
            a = aux_laws[k]
            a isa Type ? device_aux(kind, θof(r), σ, o) :
            a isa Function ? _as_aux(a(Ps[r], o), σ) : _as_aux(a, σ)
        end
    end
    aux_laws isa Function && return (r, k, o) -> _as_aux(aux_laws(Ps[r], o), σ)
    return (r, k, o) -> _as_aux(aux_laws, σ)
end

"""
    _device_ensemble(aux_laws, recordings, tts; aux_laws_blocking, artificial_noise,
                     solver_choice, solver_choice_blocking, args...)

The reference's `SamplingEnsemble(aux_laws, recordings, tts[, args]; aux_laws_blocking,
artificial_noise, solver_choice_blocking)` / `SamplingPair(…)` on the device
(src/sampling_ensemble.jl:20-40, src/sampling_pair.jl:40-50, src/sampling_unit.jl:55-66):
every keyword of those signatures is read.  `aux_laws` and `aux_laws_blocking` (default
`aux_laws`) give the laws of PP and PPb (`aux_function`), `artificial_noise` the blocking
laws' artificial observation.  `args` and the `solver_choice*` keywords select GuidedProposals'
ODE solver for the guiding term; the device's guiding term is the exact discrete filter that
every convergent solver approaches (DESIGN.md §7), so they are accepted and have no effect.
"""
function _device_ensemble(aux_laws, recordings, tts; aux_laws_blocking=nothing,
                          artificial_noise=1e-11, solver_choice=nothing,
                          solver_choice_blocking=nothing, args=nothing, pair=false, kw...)
    isempty(kw) || error("DiffusionMCMCToolsAMD: unknown keyword(s) $(collect(keys(kw)))")
    kinds = [device_model(rec.P) for rec in recordings]
    kind, _, σ = kinds[1]
    all(k -> k[1] == kind, kinds) || error("one device ensemble holds one model family")
    Ps = [rec.P for rec in recordings]
    θof = r -> kinds[r][2]
    R = length(recordings)
    recs = [(obs = [_obs(o) for o in rec.obs], x0 = rand(rec.x0_prior)) for rec in recordings]
    # the ensemble form reads a vector aux_laws / aux_laws_blocking / artificial_noise as one
    # entry per RECORDING (_vec_me, src/sampling_ensemble.jl:26-30, 44), each entry (and the pair
    # form's argument, src/sampling_pair.jl:40-50) possibly a vector per segment (aux_function);
    # the Python twin api.SamplingEnsemble._from_reference_args reads them the same way
    per_rec(v) = pair ? fill(v, R) : _vec_me(v, R)
    auxr = [aux_function(a, kind, θof, σ, Ps) for a in per_rec(aux_laws)]
    length(auxr) == R || error("aux_laws: one entry per recording ($R), got $(length(auxr))")
    aux = (r, k, o) -> auxr[r](r, k, o)
    auxb = aux
    if aux_laws_blocking !== nothing
        auxbr = [aux_function(a, kind, θof, σ, Ps) for a in per_rec(aux_laws_blocking)]
        length(auxbr) == R || error("aux_laws_blocking: one entry per recording ($R)")
        auxb = (r, k, o) -> auxbr[r](r, k, o)
    end
    noise = per_rec(artificial_noise)
    length(noise) == R && all(==(noise[1]), noise) ||
        error("artificial_noise: one value per device ensemble (the device stores one)")
    opts = DEVICE_OPTS[]
    DeviceSamplingEnsemble(kind, θof, σ, recs, tts, aux; aux_blocking=auxb,
                           artificial_noise=Float64(noise[1]), device=opts.device, seed=opts.seed)
end
_vec_me(val, N) = val isa AbstractArray ? val : fill(val, N)  # src/sampling_ensemble.jl:44

# ============================================================ views (the reference's fields)
"""
    DeviceSamplingPair(se, r)

Recording `r` (1-based) of a device ensemble, with the reference's fields `u` / `u°`
(`DeviceSamplingUnit` views, src/sampling_pair.jl:36-38): the `SamplingPair` argument of the
reference's `BiBlock(sp, range, ρ, last_block, ll_hist_len)` / `BlockCollection(sp, ranges, ρρ,
ll_hist_len)` constructors (src/biblock.jl:48-62, src/block_collection.jl:22-30).
"""
struct DeviceSamplingPair
    se::DeviceSamplingEnsemble
    r::Int
end
Base.getindex(se::DeviceSamplingEnsemble, r::Integer) = DeviceSamplingPair(se, r)

"`sp.u` / `sp.u°` of a device SamplingPair (src/sampling_unit.jl:48-53): XX, WW per segment."
struct DeviceSamplingUnit
    se::DeviceSamplingEnsemble
    r::Int
    unit::Int32
end

function Base.getproperty(sp::DeviceSamplingPair, s::Symbol)
    s === :u && return DeviceSamplingUnit(getfield(sp, :se), getfield(sp, :r), DMT_U)
    s === :u° && return DeviceSamplingUnit(getfield(sp, :se), getfield(sp, :r), DMT_UPROP)
    getfield(sp, s)
end

_segs(se::DeviceSamplingEnsemble, r) = (_seg0(se, r) + 1):(_seg0(se, r) + length(se.n_points[r]))

function Base.getproperty(u::DeviceSamplingUnit, s::Symbol)
    se = getfield(u, :se)
    if s === :XX
        return _trajectories(se, download_XX(se, getfield(u, :unit)), _segs(se, getfield(u, :r)))
    elseif s === :WW
        return _trajectories(se, download_WW(se, getfield(u, :unit)), _segs(se, getfield(u, :r)))
    end
    getfield(u, s)
end

function Base.getproperty(se::DeviceSamplingEnsemble, s::Symbol)
    # se.recordings: one SamplingPair per recording (src/sampling_ensemble.jl:17-18)
    s === :recordings && return [DeviceSamplingPair(se, r) for r in 1:length(getfield(se, :n_points))]
    getfield(se, s)
end

# the reference's constructors: device containers while use_device!(true) (the default after
# `using DiffusionMCMCToolsAMD`), the reference's CPU ones otherwise.  The reference's inner
# constructors take (aux_laws, recording(s), tts) or (…, args) (src/sampling_pair.jl:40-44,
# src/sampling_ensemble.jl:20-24): methods of arity 3 and 4.  These methods add the same two
# arities for aux_laws::Type (the tutorials pass the auxiliary law's type), strictly more
# specific than the reference's, so there is no ambiguity; the CPU fallback `invoke`s the
# reference's method of the same arity.  (Extending the reference's own constructor for its
# own argument types is type piracy, deliberately: it is what lets the tutorials' code run
# unchanged — INTEGRATION.md §2 names the explicit alternative, DeviceSamplingPair.)
function SamplingPair(aux_laws::Type, recording, tts; kw...)
    DEVICE[] || return invoke(SamplingPair, Tuple{Any,Any,Any}, aux_laws, recording, tts; kw...)
    _device_pair(aux_laws, recording, tts; kw...)
end
function SamplingPair(aux_laws::Type, recording, tts, args; kw...)
    DEVICE[] || return invoke(SamplingPair, Tuple{Any,Any,Any,Any}, aux_laws, recording, tts,
                              args; kw...)
    _device_pair(aux_laws, recording, tts; args=args, kw...)
end
# aux_laws given as laws rather than a type (a function (P, obs) -> law, one law, or a vector
# per segment; time-dependent laws included): DeviceSamplingPair / DeviceSamplingEnsemble by
# name (a method of the reference's constructor for these argument types would capture its
# CPU calls too)
DeviceSamplingPair(aux_laws, recording, tts, args...; kw...) =
    _device_pair(aux_laws, recording, tts; (isempty(args) ? () : (args=args[1],))..., kw...)
function _device_pair(aux_laws, recording, tts; kw...)
    se = _device_ensemble(aux_laws, [recording], [tts]; pair=true, kw...)
    DeviceSamplingPair(se, 1)
end

# The reference's standalone `SamplingUnit(aux_laws, recording, tts, args=tuple(); kw…)`
# (src/sampling_unit.jl:55-74): the unit `u` of a device pair built from the same arguments —
# on the device a unit is a view of its recording's paths and laws (DeviceSamplingUnit), and
# the pair's u° is held beside it unused.  Same arities and CPU fallback as SamplingPair.
# (Laws given as values rather than a type: DeviceSamplingPair(aux_laws, …).u — a method of
# DeviceSamplingUnit's own name would shadow its field constructor.)
function SamplingUnit(aux_laws::Type, recording, tts; kw...)
    DEVICE[] || return invoke(SamplingUnit, Tuple{Any,Any,Any}, aux_laws, recording, tts; kw...)
    _device_pair(aux_laws, recording, tts; kw...).u
end
function SamplingUnit(aux_laws::Type, recording, tts, args; kw...)
    DEVICE[] || return invoke(SamplingUnit, Tuple{Any,Any,Any,Any}, aux_laws, recording, tts,
                              args; kw...)
    _device_pair(aux_laws, recording, tts; args=args, kw...).u
end

function SamplingEnsemble(aux_laws::Type, recordings, tts; kw...)
    DEVICE[] || return invoke(SamplingEnsemble, Tuple{Any,Any,Any}, aux_laws, recordings, tts;
                              kw...)
    _device_ensemble(aux_laws, collect(recordings), collect(tts); kw...)
end
function SamplingEnsemble(aux_laws::Type, recordings, tts, args; kw...)
    DEVICE[] || return invoke(SamplingEnsemble, Tuple{Any,Any,Any,Any}, aux_laws, recordings,
                              tts, args; kw...)
    _device_ensemble(aux_laws, collect(recordings), collect(tts); args=args, kw...)
end
DeviceSamplingEnsemble(aux_laws, recordings::AbstractVector, tts::AbstractVector, args...; kw...) =
    _device_ensemble(aux_laws, collect(recordings), collect(tts);
                     (isempty(args) ? () : (args=args[1],))..., kw...)

# ============================================================ blocks
abstract type DeviceBlocks end

struct DeviceBlockEnsemble <: DeviceBlocks
    se::DeviceSamplingEnsemble
    layout::Int32
    b0::Int64
    b1::Int64
    hist_len::Int64
    recordings::Vector{Any}
end

struct DeviceBlockCollection <: DeviceBlocks
    se::DeviceSamplingEnsemble
    layout::Int32
    b0::Int64
    b1::Int64
    hist_len::Int64
    blocks::Vector{Any}
end

struct DeviceBiBlock{L} <: DeviceBlocks
    se::DeviceSamplingEnsemble
    layout::Int32
    b0::Int64
    b1::Int64
    hist_len::Int64
    ρ::Float64
    segs::UnitRange{Int}     # the block's segments, 1-based, global over the ensemble
end

"""
    DeviceBlock

`bb.b` / `bb.b°` of a device BiBlock (the reference's `Block{L}` views, src/block.jl:49-79):
`ll` (read and assigned), `ll_history`, `XX`, `WW` of the block's segments.
"""
struct DeviceBlock
    bb::DeviceBiBlock
    unit::Int32
end

function Base.getproperty(bb::DeviceBiBlock, s::Symbol)
    s === :b && return DeviceBlock(bb, DMT_U)
    s === :b° && return DeviceBlock(bb, DMT_UPROP)
    getfield(bb, s)
end

_llsel(b::DeviceBlock) = getfield(b, :unit) == DMT_U ? DMT_BLK_LL : DMT_BLK_LLPROP
_histsel(b::DeviceBlock) = getfield(b, :unit) == DMT_U ? DMT_BLK_LL_HIST : DMT_BLK_LLPROP_HIST

function Base.getproperty(b::DeviceBlock, s::Symbol)
    bb, unit = getfield(b, :bb), getfield(b, :unit)
    if s === :ll
        return _state(bb, _llsel(b), Float64, 1)[1]
    elseif s === :ll_history
        return vec(_hist(bb, _histsel(b), Float64))
    elseif s === :XX
        return _trajectories(bb.se, download_XX(bb.se, unit), bb.segs)
    elseif s === :WW
        return _trajectories(bb.se, download_WW(bb.se, unit), bb.segs)
    end
    getfield(b, s)
end

function Base.setproperty!(b::DeviceBlock, s::Symbol, v)
    s === :ll || error("DeviceBlock: only ll can be assigned")
    bb = getfield(b, :bb)
    vals = Float64[v]
    check(ccall((:dmt_set_block_state, libdmt), Int32,
        (Ptr{Cvoid}, Int32, Int32, Int64, Int64, Ptr{Cvoid}),
        bb.se.h, bb.layout, _llsel(b), bb.b0, bb.b1, vals))
    v
end

"""
    DeviceBlockEnsemble(se, ranges, ρρ=0.0, ll_hist_len=0)

Same arguments as `BlockEnsemble(se, ranges, ρρ, ll_hist_len)` (src/block_ensemble.jl:20):
`ranges[r]` = the 1-based segment ranges of recording r's blocks; ρρ scalar, per recording,
or per recording per block.
"""
function DeviceBlockEnsemble(se::DeviceSamplingEnsemble, ranges, ρρ=0.0, ll_hist_len=0)
    R = length(ranges)
    ll_hist_len = maximum(ll_hist_len)  # _vec_me (src/block_ensemble.jl:28): one device length
    n_blocks = Int32[length(rr) for rr in ranges]
    sf, sl, islast, rho = Int32[], Int32[], UInt8[], Float64[]
    for r in 1:R
        N = length(ranges[r])
        ρr = ρρ isa Number ? fill(ρρ, N) : (ρρ[r] isa Number ? fill(ρρ[r], N) : ρρ[r])
        for (i, rg) in enumerate(ranges[r])
            push!(sf, first(rg) - 1); push!(sl, last(rg) - 1)
            push!(islast, i == N); push!(rho, ρr[i])
        end
    end
    id = Ref{Int32}(0)
    check(ccall((:dmt_create_layout, libdmt), Int32,
        (Ptr{Cvoid}, Ptr{Int32}, Ptr{Int32}, Ptr{Int32}, Ptr{UInt8}, Ptr{Float64}, Int64,
         Ref{Int32}), se.h, n_blocks, sf, sl, islast, rho, ll_hist_len, id))
    recs = Any[]
    b = 0
    for r in 1:R
        g0 = _seg0(se, r)
        blocks = Any[DeviceBiBlock{Bool(islast[b+i])}(se, id[], b + i - 1, b + i, ll_hist_len,
                                                     rho[b+i], (g0 + sf[b+i] + 1):(g0 + sl[b+i] + 1))
                     for i in 1:n_blocks[r]]
        push!(recs, DeviceBlockCollection(se, id[], b, b + n_blocks[r], ll_hist_len, blocks))
        b += n_blocks[r]
    end
    DeviceBlockEnsemble(se, id[], 0, b, ll_hist_len, recs)
end

# The reference's constructors on device containers (same signatures): unchanged caller code
# `BlockEnsemble(se, ranges, ρ, n)` / `BlockCollection(sp, ranges, ρ, n)` /
# `BiBlock(sp, range, ρ, last, n)` builds device blocks when `se` / `sp` live on the GPU.
BlockEnsemble(se::DeviceSamplingEnsemble, ranges, ρρ=0.0, ll_hist_len=0) =
    DeviceBlockEnsemble(se, ranges, ρρ, ll_hist_len)

function BlockCollection(sp::DeviceSamplingPair, ranges, ρρ=0.0, ll_hist_len=0)
    R = length(sp.se.n_points)
    all_ranges = [r == sp.r ? collect(ranges) : UnitRange{Int}[] for r in 1:R]
    ρ = [r == sp.r ? ρρ : 0.0 for r in 1:R]
    DeviceBlockEnsemble(sp.se, all_ranges, ρ, ll_hist_len).recordings[sp.r]
end

function BiBlock(sp::DeviceSamplingPair, range::UnitRange{<:Integer}, ρ=0.0, last_block=false,
                 ll_hist_len=0)
    R = length(sp.se.n_points)
    n_blocks = Int32[r == sp.r ? 1 : 0 for r in 1:R]
    id = Ref{Int32}(0)
    check(ccall((:dmt_create_layout, libdmt), Int32,
        (Ptr{Cvoid}, Ptr{Int32}, Ptr{Int32}, Ptr{Int32}, Ptr{UInt8}, Ptr{Float64}, Int64,
         Ref{Int32}), sp.se.h, n_blocks, Int32[first(range) - 1], Int32[last(range) - 1],
        UInt8[last_block], Float64[ρ], ll_hist_len, id))
    g0 = _seg0(sp.se, sp.r)
    DeviceBiBlock{Bool(last_block)}(sp.se, id[], 0, 1, ll_hist_len, ρ,
                                    (g0 + first(range)):(g0 + last(range)))
end

"""
    Block(u::DeviceSamplingUnit, range, last_block=false, ll_hist_len=0)

The reference's standalone `Block(u, range, last_block, ll_hist_len)` (src/block.jl:60-79): the
window `range` (1-based segments of u's recording) of one unit.  On the device a block's state
lives in a layout of the pair (its ll, history, and the views of u's and u°'s paths and laws),
so this is the `b` (u) or `b°` (u°) view of a one-block device BiBlock over `range` with ρ = 0:
`ll` starts at −Inf (src/block.jl:75), and `loglikhd!`, `recompute_path!(b, WW)`,
`find_W_for_X!`, `set_ll!` / `save_ll!` act on that unit only.
"""
function Block(u::DeviceSamplingUnit, range::UnitRange{<:Integer}, last_block=false,
               ll_hist_len=0)
    bb = BiBlock(DeviceSamplingPair(u.se, u.r), range, 0.0, last_block, ll_hist_len)
    DeviceBlock(bb, u.unit)
end

_n(x::DeviceBlocks) = x.b1 - x.b0

# ---- imputation and MH (src/biblock.jl:78-127, block_collection.jl:46-68, block_ensemble.jl:50-69)
sync(x::DeviceBlocks) = sync(x.se)

"""
    draw_proposal_path!(x; Z=nothing, iter=nothing, salt=nothing)

pCN proposal under the accepted law into u°.  With no keyword the normals are the next ones of
the device stream counter (every call fresh, as the reference's `rand!` on the global RNG);
`iter`/`salt` select a reproducible keyed stream; `Z` supplies them (parity mode).
"""
function draw_proposal_path!(x::DeviceBlocks; Z=nothing, iter=nothing, salt=nothing)
    iter, salt = _key(iter, salt)
    pz = Z === nothing ? Ptr{Float64}(C_NULL) : pointer(Z)
    # no success buffer: the draw may be deferred and fused with the accept_reject_proposal_path!
    # that follows (include/dmt.h, deferred draws); the flags are read only if used
    GC.@preserve Z check(ccall((:dmt_draw_proposal, libdmt), Int32,
        (Ptr{Cvoid}, Int32, Int64, Int64, Ptr{Float64}, Int64, UInt32, Ptr{UInt8}),
        x.se.h, x.layout, x.b0, x.b1, pz, iter, salt, Ptr{UInt8}(C_NULL)))
    DrawSuccess(x)
end

"""
    DrawSuccess

What `draw_proposal_path!` returns (the reference returns the success flag(s),
src/biblock.jl:78-92): read from the device (dmt_draw_success) only when used — `Bool(s)`,
`s[i]`, `collect(s)`, `all(s)`, `s == v` — so an unused return value costs nothing.
"""
struct DrawSuccess{X}
    x::X
end
function _flags(s::DrawSuccess)
    x = s.x
    ok = Vector{UInt8}(undef, _n(x))
    check(ccall((:dmt_draw_success, libdmt), Int32, (Ptr{Cvoid}, Int32, Int64, Int64, Ptr{UInt8}),
                x.se.h, x.layout, x.b0, x.b1, ok))
    Bool.(ok)
end
Base.Bool(s::DrawSuccess) = all(_flags(s))
Base.convert(::Type{Bool}, s::DrawSuccess) = Bool(s)
Base.collect(s::DrawSuccess) = _flags(s)
Base.getindex(s::DrawSuccess, i...) = _flags(s)[i...]
Base.all(s::DrawSuccess) = all(_flags(s))
Base.:(==)(s::DrawSuccess, v) = (s.x isa DeviceBiBlock ? Bool(s) : _flags(s)) == v

"draw_proposal_path!(u::SamplingUnit) (src/sampling_unit.jl:118-120): (success, ll)."
function draw_proposal_path!(u::DeviceSamplingUnit)
    ok, ll = draw_unit!(u.se, u.unit, u.r - 1, u.r)
    ok[1], ll[1]
end

function accept_reject_proposal_path!(x::DeviceBlocks, mcmciter; E=nothing, salt=nothing)
    salt = salt === nothing ? DMT_RNG_AUTO : UInt32(salt)
    acc = Vector{UInt8}(undef, _n(x))
    pe = E === nothing ? Ptr{Float64}(C_NULL) : pointer(E)
    GC.@preserve E check(ccall((:dmt_accept_reject, libdmt), Int32,
        (Ptr{Cvoid}, Int32, Int64, Int64, Ptr{Float64}, Int64, UInt32, Ptr{UInt8}),
        x.se.h, x.layout, x.b0, x.b1, pe, mcmciter, salt, acc))
    nothing
end

# fused iterations: a BlockEnsemble's sums are over every rank (collective); a collection's or
# a block's are this rank's (the _local entry points: no collective)
"draw_proposal_path! + accept_reject_proposal_path!(·, i) + (fetch_ll, fetch_ll°, #accepted)."
function mcmc_step!(x::DeviceBlocks, mcmciter; salt=nothing)
    salt = salt === nothing ? DMT_RNG_AUTO : UInt32(salt)
    a, b, n = Ref(0.0), Ref(0.0), Ref{Int64}(0)
    if x isa DeviceBlockEnsemble
        check(ccall((:dmt_mcmc_step, libdmt), Int32,
            (Ptr{Cvoid}, Int32, Int64, Int64, Int64, UInt32, Ref{Float64}, Ref{Float64}, Ref{Int64}),
            x.se.h, x.layout, x.b0, x.b1, mcmciter, salt, a, b, n))
    else
        check(ccall((:dmt_mcmc_step_local, libdmt), Int32,
            (Ptr{Cvoid}, Int32, Int64, Int64, Int64, UInt32, Ref{Float64}, Ref{Float64}, Ref{Int64}),
            x.se.h, x.layout, x.b0, x.b1, mcmciter, salt, a, b, n))
    end
    a[], b[], n[]
end

"n_iter iterations of mcmc_step! from iter0 on, no host round trips; (n_iter, 3) results."
function mcmc_run!(x::DeviceBlocks, iter0, n_iter; salt=nothing)
    salt = salt === nothing ? DMT_RNG_AUTO : UInt32(salt)
    out = Matrix{Float64}(undef, 3, n_iter)
    if x isa DeviceBlockEnsemble
        check(ccall((:dmt_mcmc_run, libdmt), Int32,
            (Ptr{Cvoid}, Int32, Int64, Int64, Int64, Int64, UInt32, Ptr{Float64}),
            x.se.h, x.layout, x.b0, x.b1, iter0, n_iter, salt, out))
    else
        check(ccall((:dmt_mcmc_run_local, libdmt), Int32,
            (Ptr{Cvoid}, Int32, Int64, Int64, Int64, Int64, UInt32, Ptr{Float64}),
            x.se.h, x.layout, x.b0, x.b1, iter0, n_iter, salt, out))
    end
    permutedims(out)
end

# ---- log-likelihoods (src/block.jl:138-152; biblock.jl:240,248; block_collection.jl:166-197)
_ll!(x, unit) = check(ccall((:dmt_loglikhd, libdmt), Int32,
    (Ptr{Cvoid}, Int32, Int32, Int64, Int64), x.se.h, x.layout, unit, x.b0, x.b1))
loglikhd!(x::DeviceBlocks) = _ll!(x, DMT_U)
loglikhd°!(x::DeviceBlocks) = _ll!(x, DMT_UPROP)
loglikhd!(b::DeviceBlock) = _ll!(getfield(b, :bb), getfield(b, :unit))

"GP.loglikhd(u::SamplingUnit) (src/sampling_unit.jl:109): the stored path's log-likelihood."
function GP.loglikhd(u::DeviceSamplingUnit)
    # the handle's internal layout 0 holds one terminal block per recording over all segments
    check(ccall((:dmt_loglikhd, libdmt), Int32, (Ptr{Cvoid}, Int32, Int32, Int64, Int64),
                u.se.h, 0, u.unit, u.r - 1, u.r))
    out = Vector{Float64}(undef, 1)
    check(ccall((:dmt_get_block_state, libdmt), Int32,
        (Ptr{Cvoid}, Int32, Int32, Int64, Int64, Ptr{Cvoid}),
        u.se.h, 0, u.unit == DMT_U ? DMT_BLK_LL : DMT_BLK_LLPROP, u.r - 1, u.r, out))
    out[1]
end

# fetch_ll(be) is the whole (multi-GPU) ensemble's (a collective over ranks); a collection's or
# a block's is this rank's (src/block_collection.jl:144,156, src/block_ensemble.jl:140,152)
function _fetch(x::DeviceBlocks)
    a, b, n = Ref(0.0), Ref(0.0), Ref{Int64}(0)
    if x isa DeviceBlockEnsemble
        check(ccall((:dmt_fetch_ll, libdmt), Int32,
            (Ptr{Cvoid}, Int32, Int64, Int64, Int64, Ref{Float64}, Ref{Float64}, Ref{Int64}),
            x.se.h, x.layout, x.b0, x.b1, 0, a, b, n))
    else
        check(ccall((:dmt_fetch_ll_local, libdmt), Int32,
            (Ptr{Cvoid}, Int32, Int64, Int64, Int64, Ref{Float64}, Ref{Float64}, Ref{Int64}),
            x.se.h, x.layout, x.b0, x.b1, 0, a, b, n))
    end
    a[], b[]
end
fetch_ll(x::DeviceBlocks) = _fetch(x)[1]
fetch_ll°(x::DeviceBlocks) = _fetch(x)[2]

"recompute_path!(bb.b°, bb.b.WW; skip) over the blocks (src/block.jl:159-187)."
function recompute_path!(x::DeviceBlocks; skip=0)
    ok = Vector{UInt8}(undef, _n(x))
    check(ccall((:dmt_recompute_path, libdmt), Int32,
        (Ptr{Cvoid}, Int32, Int64, Int64, Int32, Ptr{UInt8}),
        x.se.h, x.layout, x.b0, x.b1, skip, ok))
    Bool.(ok)
end
# the reference's own call form, recompute_path!(bb.b°, bb.b.WW; skip) (src/biblock.jl:343):
# the device re-solves b° with b's Wiener path, the only one the reference passes
function recompute_path!(b::DeviceBlock, WW; skip=0)
    getfield(b, :unit) == DMT_UPROP ||
        error("recompute_path!: the device re-solves the proposal bb.b° with bb.b.WW")
    recompute_path!(getfield(b, :bb); skip=skip)
end

"""
    GP.equalize_obs_params!(x)

src/biblock.jl:375-387: u°'s observation parameters ← u's.  The device stores a recording's
observations once for both u and u° (`upload_obs!`), so they never differ: nothing to copy, no
critical change.
"""
GP.equalize_obs_params!(x::DeviceBlocks) = false

"Observation information at every segment end (packed H, F, c) + artificial noise."
upload_obs!(se::DeviceSamplingEnsemble, Hobs, Fobs, cobs; artificial_noise=1e-11) =
    GC.@preserve Hobs Fobs cobs check(ccall((:dmt_upload_obs, libdmt), Int32,
        (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Float64),
        se.h, Hobs, Fobs, cobs, artificial_noise))

"GP.set_obs!(bb) (src/biblock.jl:273-280, broadcasts src/block_collection.jl:198, src/block_ensemble.jl:192)."
GP.set_obs!(x::DeviceBlocks) = check(ccall((:dmt_set_obs, libdmt), Int32,
    (Ptr{Cvoid}, Int32, Int64, Int64), x.se.h, x.layout, x.b0, x.b1))

_rgt!(x::DeviceBlocks, unit) = check(ccall(
    (:dmt_recompute_guiding_term, libdmt), Int32, (Ptr{Cvoid}, Int32, Int64, Int64, Int32),
    x.se.h, x.layout, x.b0, x.b1, unit))
"""
    GP.recompute_guiding_term!(x, [::Val{:P_only} | ::Val{:P°_only}])

GP.recompute_guiding_term! on the device: of a BiBlock / collection / ensemble with no flag both
the accepted and the proposal laws, b then b° (src/biblock.jl:288-291,
src/block_collection.jl:208-210); `Val(:P_only)` the accepted laws, `Val(:P°_only)` the proposal
laws (src/block_collection.jl:212-221); of a block view `bb.b` / `bb.b°` its own laws
(src/block.jl:102-110, as `(bb->recompute_guiding_term!(bb.b)).(B)` in
docs/src/tutorials/biblock/smoothing_with_blocking.md:38); of a SamplingUnit its PP over the
whole recording (src/sampling_unit.jl:100-102).
"""
GP.recompute_guiding_term!(x::DeviceBlocks) = (_rgt!(x, DMT_U); _rgt!(x, DMT_UPROP))
GP.recompute_guiding_term!(x::DeviceBlocks, ::Val{:P_only}) = _rgt!(x, DMT_U)
GP.recompute_guiding_term!(x::DeviceBlocks, ::Val{:P°_only}) = _rgt!(x, DMT_UPROP)
GP.recompute_guiding_term!(b::DeviceBlock) = _rgt!(getfield(b, :bb), getfield(b, :unit))
GP.recompute_guiding_term!(u::DeviceSamplingUnit) = check(ccall(
    (:dmt_recompute_guiding_term, libdmt), Int32, (Ptr{Cvoid}, Int32, Int64, Int64, Int32),
    u.se.h, 0, u.r - 1, u.r, u.unit))

# ---- parameter names (src/param_names_collections.jl) for device blocks: only the θ° → name
# maps `updt` are needed (the device re-derives the auxiliary laws from θ itself)
_pn_unit(θnames, pdep) = (var = (), var_aux = [],
    updt = Tuple(findfirst(==(p[1]), θnames) => p[2] for p in pdep if p[1] in θnames),
    updt_aux = [], updt_obs = [])
_pn_block(θnames, pdep) = (PP = _pn_unit(θnames, pdep), P_last = _pn_unit(θnames, pdep),
    P_excl = _pn_unit(θnames, pdep), Pb_excl = _pn_unit(θnames, pdep))
"ParamNamesBlock(b, θnames, pdep, odeps) of a device block view (src/param_names_collections.jl:204-225)."
ParamNamesBlock(b::DeviceBlock, θnames, pdep, odeps) = _pn_block(θnames, pdep)
"ParamNamesRecording(bc, θnames, pdep, odeps) of a device BlockCollection (src/param_names_collections.jl:249-257)."
ParamNamesRecording(bc::DeviceBlockCollection, θnames, pdep, odeps) =
    (blocks = [_pn_block(θnames, pdep) for _ in bc.blocks],)
"ParamNamesAllObs(be, θnames, all_obs) of a device BlockEnsemble (src/param_names_collections.jl:274-288)."
ParamNamesAllObs(be::DeviceBlockEnsemble, θnames, all_obs) =
    (recordings = [ParamNamesRecording(be.recordings[i], θnames, all_obs.param_depend_rev[i],
                                       all_obs.obs_depend_rev[i]) for i in 1:length(be.recordings)],)

const _PAR_NAMES = Dict(
    DMT_MODEL_FHN => Dict(:ϵ => 0, :s => 1, :γ => 2, :β => 3, :σ => 4),
    DMT_MODEL_LORENZ => Dict(:s => 0, :r => 1, :β => 2))

"The θ° entry → device parameter index map of one block's pnames (all four law collections)."
function _param_map(se::DeviceSamplingEnsemble, pnames_block)
    names = get(_PAR_NAMES, se.model, Dict{Symbol,Int}())
    m = Dict{Int32,Int}()
    for coll in (:PP, :P_last, :P_excl, :Pb_excl)
        u = getproperty(pnames_block, coll)
        # observation parameters (DD.set_parameters!(PP, θ°, updt, updt_aux, updt_obs),
        # src/biblock.jl:373-375) are not device state: refuse instead of dropping them
        hasproperty(u, :updt_obs) && any(!isempty, u.updt_obs) &&
            error("set_proposal_law!: observation parameters (updt_obs) are not updated on the device")
        pairs = collect(u.updt)
        for ua in u.updt_aux
            append!(pairs, collect(ua))
        end
        for (idx, name) in pairs
            k = Int32(name isa Symbol ? names[name] : name)
            get(m, k, idx) == idx || error("parameter $name updated from two entries of θ°")
            m[k] = idx
        end
    end
    m
end

# critical_change: nothing (the reference's default, GP.is_critical_update) → -1, recompute the
# guiding term where the auxiliary law changed; true → 1, every block; false → 0, only where
# equalizing u°'s law with u's changed it (dmt_set_proposal_law_cc, include/dmt.h)
_cc(c) = c === nothing ? Int32(-1) : (c ? Int32(1) : Int32(0))

function _set_law!(x::DeviceBlocks, θ°, pmap, cc::Int32; skip=0)
    idx = collect(keys(pmap))
    val = Float64[θ°[pmap[k]] for k in idx]
    ok = Vector{UInt8}(undef, _n(x))
    crit = Vector{UInt8}(undef, _n(x))
    check(ccall((:dmt_set_proposal_law_cc, libdmt), Int32,
        (Ptr{Cvoid}, Int32, Int64, Int64, Int32, Ptr{Int32}, Ptr{Float64}, Int32, Int32,
         Ptr{UInt8}, Ptr{UInt8}), x.se.h, x.layout, x.b0, x.b1, length(idx), idx, val, skip, cc,
        ok, crit))
    Bool.(ok)
end

"""
    set_proposal_law!(x, θ°, pnames, critical_change=nothing; skip=0)

The reference's `set_proposal_law!` (src/biblock.jl:334-344, src/block_collection.jl:264-276,
src/block_ensemble.jl:242-255) on device blocks: `pnames` as the reference's (a BiBlock's
NamedTuple / ParamNamesBlock of `PP, P_last, P_excl, Pb_excl` with `updt` pairs `idx => name`;
`pnames.blocks[i]` of a collection; `pnames.recordings[r].blocks[i]` of an ensemble).  u°'s laws
← u's with the named parameters set from θ°, the guiding term of b° recomputed — omitted
(the reference's default GP.is_critical_update): where the auxiliary law changed (an unchanged
law's recomputation reproduces its guiding term bit for bit); `true`: every block; `false`: only
where equalizing b°'s law with b's changed it (:340-342, 361-362); a collection / ensemble also
takes one Bool per block (per recording a vector) — then recompute_path!(b°, b.WW; skip).  One
ccall over all blocks whose maps and flags agree.
"""
function set_proposal_law!(bb::DeviceBiBlock, θ°, pnames, critical_change=nothing; skip=0)
    _set_law!(bb, θ°, _param_map(bb.se, pnames), _cc(critical_change); skip=skip)
end

function _set_law_blocks!(x, blocks, pblocks, θ°, critical_change; skip=0)
    maps = [_param_map(x.se, pb) for pb in pblocks]
    ccs = critical_change isa AbstractArray ?
        Int32[_cc(c) for c in Iterators.flatten(critical_change)] :
        fill(_cc(critical_change), length(blocks))
    length(ccs) == length(blocks) || error("critical_change: $(length(ccs)) flags for $(length(blocks)) blocks")
    all(==(maps[1]), maps) && all(==(ccs[1]), ccs) && return _set_law!(x, θ°, maps[1], ccs[1]; skip=skip)
    reduce(vcat, [_set_law!(bb, θ°, m, c; skip=skip) for (bb, m, c) in zip(blocks, maps, ccs)])
end

set_proposal_law!(bc::DeviceBlockCollection, θ°, pnames, critical_change=nothing; skip=0) =
    _set_law_blocks!(bc, bc.blocks, pnames.blocks, θ°, critical_change; skip=skip)

set_proposal_law!(be::DeviceBlockEnsemble, θ°, pnames, critical_change=nothing; skip=0) =
    _set_law_blocks!(be, [bb for bc in be.recordings for bb in bc.blocks],
                     [pb for pr in pnames.recordings for pb in pr.blocks], θ°, critical_change;
                     skip=skip)

"find_W_for_X!(b) (src/block.jl:118-131): u.WW from u.XX under the accepted laws."
find_W_for_X!(x::DeviceBlocks) = check(ccall((:dmt_find_W_for_X, libdmt), Int32,
    (Ptr{Cvoid}, Int32, Int64, Int64), x.se.h, x.layout, x.b0, x.b1))
find_W_for_X!(b::DeviceBlock) = find_W_for_X!(getfield(b, :bb))

# ---- swaps, histories (src/biblock.jl:135-259)
_swap!(x, what) = check(ccall((:dmt_swap, libdmt), Int32,
    (Ptr{Cvoid}, Int32, Int32, Int64, Int64), x.se.h, x.layout, what, x.b0, x.b1))
swap_paths!(x::DeviceBlocks) = _swap!(x, DMT_SWAP_XX | DMT_SWAP_WW)
swap_XX!(x::DeviceBlocks) = _swap!(x, DMT_SWAP_XX)
swap_WW!(x::DeviceBlocks) = _swap!(x, DMT_SWAP_WW)
swap_PP!(x::DeviceBlocks) = _swap!(x, DMT_SWAP_PP)
swap_ll!(x::DeviceBlocks) = _swap!(x, DMT_SWAP_LL)

save_ll!(x::DeviceBlocks, i::Integer) = check(ccall((:dmt_save_ll, libdmt), Int32,
    (Ptr{Cvoid}, Int32, Int64, Int64, Int64), x.se.h, x.layout, x.b0, x.b1, i))
"save_ll!(b, i) of a block view (src/block.jl:94): ll_history[i] = ll."
save_ll!(b::DeviceBlock, i::Integer) = set_ll!(b, i, b.ll)

"set_ll!(b, i, v) (src/block.jl:82-86): ll_history[i] of bb.b (unit DMT_U) or bb.b°."
function set_ll!(x::DeviceBlocks, i::Integer, v; unit=DMT_U)
    vals = Vector{Float64}(undef, x.b1 - x.b0)
    vals .= v
    check(ccall((:dmt_set_ll, libdmt), Int32,
                (Ptr{Cvoid}, Int32, Int32, Int64, Int64, Int64, Ptr{Float64}),
                x.se.h, x.layout, unit, x.b0, x.b1, i, vals))
end
set_ll!(b::DeviceBlock, i::Integer, v) = set_ll!(getfield(b, :bb), i, v; unit=getfield(b, :unit))

function set_accepted!(x::DeviceBlocks, i::Integer, v)
    vv = fill(UInt8(v), _n(x))
    check(ccall((:dmt_set_accepted, libdmt), Int32,
        (Ptr{Cvoid}, Int32, Int64, Int64, Int64, Ptr{UInt8}), x.se.h, x.layout, x.b0, x.b1, i, vv))
end

function _state(x::DeviceBlocks, what, T, dims...)
    out = Array{T}(undef, dims...)
    check(ccall((:dmt_get_block_state, libdmt), Int32,
        (Ptr{Cvoid}, Int32, Int32, Int64, Int64, Ptr{Cvoid}),
        x.se.h, x.layout, what, x.b0, x.b1, out))
    out
end
# histories come back iteration-major: [hist_len][nblocks] == Julia (nblocks, hist_len)
_hist(x, what, T) = _state(x, what, T, _n(x), x.hist_len)

function ll_of_accepted(x::DeviceBlocks, i)
    acc = _hist(x, DMT_BLK_ACC_HIST, UInt8)[:, i] .!= 0
    llh = _hist(x, DMT_BLK_LL_HIST, Float64)[:, i]
    llph = _hist(x, DMT_BLK_LLPROP_HIST, Float64)[:, i]
    v = ifelse.(acc, llph, llh)
    x isa DeviceBiBlock ? v[1] : v
end

function accpt_rate(x::DeviceBlocks, range)
    acc = _hist(x, DMT_BLK_ACC_HIST, UInt8)[:, range] .!= 0
    v = vec(sum(acc; dims=2)) ./ length(range)
    x isa DeviceBiBlock ? v[1] : v
end

end # module
