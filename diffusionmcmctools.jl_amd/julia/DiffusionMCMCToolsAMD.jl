#= DiffusionMCMCToolsAMD — Julia binding of libdmt (include/dmt.h) for DiffusionMCMCTools.jl.

Device-resident counterparts of SamplingEnsemble / BlockEnsemble / BlockCollection / BiBlock
whose methods carry the reference's names and argument meaning, each one `ccall` over a block
range.  The host arrays passed in are the reference's own containers reinterpreted
(Vector{SVector{d,Float64}} == double[npts][d]).

No Julia toolchain exists in the build image, so this file is shipped as source and is not
exercised by the test suite; the Python mirror (../api.py) calls the same entry points and is
tested.  See INTEGRATION.md for the wiring into the reference package.
=#
module DiffusionMCMCToolsAMD

using StaticArrays
using LinearAlgebra: I, det, inv

import DiffusionMCMCTools: draw_proposal_path!, accept_reject_proposal_path!, loglikhd!,
    loglikhd°!, fetch_ll, fetch_ll°, save_ll!, set_ll!, set_accepted!, swap_paths!, swap_XX!,
    swap_WW!, swap_PP!, swap_ll!, ll_of_accepted, accpt_rate, recompute_path!, find_W_for_X!,
    BiBlock, BlockCollection, BlockEnsemble

export DeviceSamplingEnsemble, DeviceBlockEnsemble, DeviceBlockCollection, DeviceBiBlock,
    mcmc_step!, mcmc_run!, download_XX, download_WW, upload_obs!, set_obs!,
    recompute_guiding_term!, set_proposal_law!, snapshot_every!, equalize_obs_params!,
    law_record, guiding_linear

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
        se = new(h[], Int32(model), d, m, [collect(Int, r) for r in n_points], sum(npts))
        finalizer(se) do x
            x.h == C_NULL || ccall((:dmt_destroy, libdmt), Int32, (Ptr{Cvoid},), x.h)
            x.h = C_NULL
        end
        se
    end
end

"Concatenate per-segment trajectories (Vector{SVector}) recording-major into one flat buffer."
flatten_paths(segs) = reduce(vcat, (collect(reinterpret(Float64, s)) for s in segs))

upload_grid!(se::DeviceSamplingEnsemble, t::Vector{Float64}) =
    check(ccall((:dmt_upload_grid, libdmt), Int32, (Ptr{Cvoid}, Ptr{Float64}), se.h, t))

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
    law_record(θrec, σ, B̃, β̃, σ̃, c0; anchor=nothing)

One segment's law record (DMT_LAW_STRIDE doubles, include/dmt.h): θrec = the target's
parameters in the device order (OU: Θ row-major at 1:d², μ at 10:9+d; FHN: 1/ϵ, s, γ, β, ϵ, σ;
Lorenz: s, r, β), σ (d×m), the auxiliary law's B̃, β̃, σ̃, c(t₀), and the linearisation point
of a linearised auxiliary law (FitzHughNagumoAux: y_T; Lorenz: x_T).
"""
function law_record(θrec, σ::AbstractMatrix, B̃::AbstractMatrix, β̃, σ̃::AbstractMatrix, c0;
                    anchor=nothing)
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
    rec
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

"Information (H, F, c) of an observation v ~ N(L x, Σ) (ObservationSchemes LinearGsnObs)."
function obs_info(v, L::AbstractMatrix, Σ::AbstractMatrix)
    Si = inv(Σ)
    H, F = L' * Si * L, L' * Si * v
    H, F, 0.5 * v' * Si * v + 0.5 * length(v) * log(2π) + 0.5 * log(det(Σ))
end

"""
    DeviceSamplingEnsemble(model, θrec, σ, recordings, tts, aux; artificial_noise=1e-11,
                           blocking=true, kw...)

`SamplingEnsemble(aux_laws, recordings, tts; artificial_noise)` on the device:
`recordings[r] = (obs = [(t, v, L, Σ), …], x0 = …)`, `tts[r][k]` the grid of segment k,
`aux(r, k, obs) -> (B̃, β̃, σ̃, anchor)` the auxiliary law of segment k (e.g. FitzHughNagumoAux
linearised at the observed y: `(DD.B(t0, P̃), DD.β(t0, P̃), DD.σ(t0, x, P̃), yT)`).  Guiding terms
through each recording's segments (build_guid_prop), blocking laws with an exact full-state
artificial end observation (guid_prop_for_blocking; a placeholder until set_obs!), the
observations for the device's re-derivations, then init_paths! from x0.
"""
function DeviceSamplingEnsemble(model::Integer, θrec, σ::AbstractMatrix, recordings, tts, aux;
                                artificial_noise=1e-11, blocking=true, kw...)
    d, m = size(σ)
    t_all, H_all, F_all, laws, infos = Float64[], Matrix{Float64}[], Matrix{Float64}[], Vector{Float64}[], Any[]
    Hb_all, Fb_all, lawsb = Matrix{Float64}[], Matrix{Float64}[], Vector{Float64}[]
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
            B̃, β̃, σ̃, _ = auxes[k]
            H, F, c = guiding_linear(B̃, β̃, σ̃, Float64.(tts[r][k]), HT, FT, cT)
            chain[k] = (H, F, c)
            nxt = (H[1, :], F[1, :], c[1])
        end
        for k in 1:K
            B̃, β̃, σ̃, an = auxes[k]
            append!(t_all, tts[r][k]); push!(H_all, chain[k][1]); push!(F_all, chain[k][2])
            push!(laws, law_record(θrec, σ, B̃, β̃, σ̃, chain[k][3][1]; anchor=an))
            push!(infos, info[k])
            if blocking
                v = zeros(d); vo = collect(rec.obs[k].v); v[1:min(d, length(vo))] .= vo[1:min(d, length(vo))]
                Ha, Fa, ca = obs_info(v, Matrix(1.0I, d, d), artificial_noise * Matrix(1.0I, d, d))
                Ho, Fo, co = info[k]
                H, F, c = guiding_linear(B̃, β̃, σ̃, Float64.(tts[r][k]), Ha + Ho, Fa + Fo, ca + co)
                push!(Hb_all, H); push!(Fb_all, F)
                push!(lawsb, law_record(θrec, σ, B̃, β̃, σ̃, c[1]; anchor=an))
            end
        end
        push!(n_points, [length(g) for g in tts[r]])
    end
    se = DeviceSamplingEnsemble(model, d, m, n_points; kw...)
    upload_grid!(se, t_all)
    flat(Ms) = vec(permutedims(reduce(vcat, Ms)))     # point-major, components contiguous
    upload_law!(se, DMT_U, DMT_LAW_PP, flat(H_all), flat(F_all), reduce(vcat, laws))
    blocking && upload_law!(se, DMT_U, DMT_LAW_PPB, flat(Hb_all), flat(Fb_all), reduce(vcat, lawsb))
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
end

"""
    DeviceSamplingPair(se, r)

Recording `r` (1-based) of a device ensemble: the `SamplingPair` argument of the reference's
`BiBlock(sp, range, ρ, last_block, ll_hist_len)` / `BlockCollection(sp, ranges, ρρ,
ll_hist_len)` constructors (src/biblock.jl:48-62, src/block_collection.jl:22-30).
"""
struct DeviceSamplingPair
    se::DeviceSamplingEnsemble
    r::Int
end
Base.getindex(se::DeviceSamplingEnsemble, r::Integer) = DeviceSamplingPair(se, r)

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
        blocks = Any[DeviceBiBlock{Bool(islast[b+i])}(se, id[], b + i - 1, b + i, ll_hist_len,
                                                     rho[b+i]) for i in 1:n_blocks[r]]
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

function BiBlock(sp::DeviceSamplingPair, range::UnitRange{Int64}, ρ=0.0, last_block=false,
                 ll_hist_len=0)
    R = length(sp.se.n_points)
    n_blocks = Int32[r == sp.r ? 1 : 0 for r in 1:R]
    id = Ref{Int32}(0)
    check(ccall((:dmt_create_layout, libdmt), Int32,
        (Ptr{Cvoid}, Ptr{Int32}, Ptr{Int32}, Ptr{Int32}, Ptr{UInt8}, Ptr{Float64}, Int64,
         Ref{Int32}), sp.se.h, n_blocks, Int32[first(range) - 1], Int32[last(range) - 1],
        UInt8[last_block], Float64[ρ], ll_hist_len, id))
    DeviceBiBlock{Bool(last_block)}(sp.se, id[], 0, 1, ll_hist_len, ρ)
end

_n(x::DeviceBlocks) = x.b1 - x.b0

# ---- imputation and MH (src/biblock.jl:78-127, block_collection.jl:46-68, block_ensemble.jl:50-69)
"""
    draw_proposal_path!(x; Z=nothing, iter=nothing, salt=nothing)

pCN proposal under the accepted law into u°.  With no keyword the normals are the next ones of
the device stream counter (every call fresh, as the reference's `rand!` on the global RNG);
`iter`/`salt` select a reproducible keyed stream; `Z` supplies them (parity mode).
"""
function draw_proposal_path!(x::DeviceBlocks; Z=nothing, iter=nothing, salt=nothing)
    iter, salt = _key(iter, salt)
    ok = Vector{UInt8}(undef, _n(x))
    pz = Z === nothing ? Ptr{Float64}(C_NULL) : pointer(Z)
    GC.@preserve Z check(ccall((:dmt_draw_proposal, libdmt), Int32,
        (Ptr{Cvoid}, Int32, Int64, Int64, Ptr{Float64}, Int64, UInt32, Ptr{UInt8}),
        x.se.h, x.layout, x.b0, x.b1, pz, iter, salt, ok))
    x isa DeviceBiBlock ? Bool(ok[1]) : Bool.(ok)
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

"draw_proposal_path! + accept_reject_proposal_path!(·, i) + (fetch_ll, fetch_ll°, #accepted)."
function mcmc_step!(x::DeviceBlocks, mcmciter; salt=nothing)
    salt = salt === nothing ? DMT_RNG_AUTO : UInt32(salt)
    a, b, n = Ref(0.0), Ref(0.0), Ref{Int64}(0)
    check(ccall((:dmt_mcmc_step, libdmt), Int32,
        (Ptr{Cvoid}, Int32, Int64, Int64, Int64, UInt32, Ref{Float64}, Ref{Float64}, Ref{Int64}),
        x.se.h, x.layout, x.b0, x.b1, mcmciter, salt, a, b, n))
    a[], b[], n[]
end

"n_iter iterations of mcmc_step! from iter0 on, no host round trips; (n_iter, 3) results."
function mcmc_run!(x::DeviceBlocks, iter0, n_iter; salt=nothing)
    salt = salt === nothing ? DMT_RNG_AUTO : UInt32(salt)
    out = Matrix{Float64}(undef, 3, n_iter)
    check(ccall((:dmt_mcmc_run, libdmt), Int32,
        (Ptr{Cvoid}, Int32, Int64, Int64, Int64, Int64, UInt32, Ptr{Float64}),
        x.se.h, x.layout, x.b0, x.b1, iter0, n_iter, salt, out))
    permutedims(out)
end

# ---- log-likelihoods (src/block.jl:138-152; biblock.jl:240,248; block_collection.jl:166-197)
_ll!(x, unit) = check(ccall((:dmt_loglikhd, libdmt), Int32,
    (Ptr{Cvoid}, Int32, Int32, Int64, Int64), x.se.h, x.layout, unit, x.b0, x.b1))
loglikhd!(x::DeviceBlocks) = _ll!(x, DMT_U)
loglikhd°!(x::DeviceBlocks) = _ll!(x, DMT_UPROP)

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

"""
    GP.equalize_obs_params!(x)

src/biblock.jl:375-387: u°'s observation parameters ← u's.  The device stores a recording's
observations once for both u and u° (`upload_obs!`), so they never differ: nothing to copy, no
critical change.
"""
equalize_obs_params!(x::DeviceBlocks) = falses(_n(x))

"Observation information at every segment end (packed H, F, c) + artificial noise."
upload_obs!(se::DeviceSamplingEnsemble, Hobs, Fobs, cobs; artificial_noise=1e-11) =
    GC.@preserve Hobs Fobs cobs check(ccall((:dmt_upload_obs, libdmt), Int32,
        (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Float64),
        se.h, Hobs, Fobs, cobs, artificial_noise))

"GP.set_obs!(bb) (src/biblock.jl:273-280) over the blocks."
set_obs!(x::DeviceBlocks) = check(ccall((:dmt_set_obs, libdmt), Int32,
    (Ptr{Cvoid}, Int32, Int64, Int64), x.se.h, x.layout, x.b0, x.b1))

_rgt!(x::DeviceBlocks, unit) = check(ccall(
    (:dmt_recompute_guiding_term, libdmt), Int32, (Ptr{Cvoid}, Int32, Int64, Int64, Int32),
    x.se.h, x.layout, x.b0, x.b1, unit))
"""
    recompute_guiding_term!(x, [::Val{:P_only} | ::Val{:P°_only}])

GP.recompute_guiding_term! on the device: with no flag both the accepted and the proposal laws,
b then b° (src/biblock.jl:288-291, src/block_collection.jl:208-210); `Val(:P_only)` the
accepted laws (= `recompute_guiding_term!(bb.b)`), `Val(:P°_only)` the proposal laws
(src/block_collection.jl:212-221).
"""
recompute_guiding_term!(x::DeviceBlocks) = (_rgt!(x, DMT_U); _rgt!(x, DMT_UPROP))
recompute_guiding_term!(x::DeviceBlocks, ::Val{:P_only}) = _rgt!(x, DMT_U)
recompute_guiding_term!(x::DeviceBlocks, ::Val{:P°_only}) = _rgt!(x, DMT_UPROP)

"""
    set_proposal_law!(x, θ°::AbstractVector, pnames::AbstractVector{Symbol}; skip=0)

set_proposal_law! (src/biblock.jl:334-345) on the device: u°'s laws ← u's with the named
parameters set to θ° (names as DiffusionDefinition's: FHN `:ϵ, :s, :γ, :β, :σ`, Lorenz
`:s, :r, :β`), the guiding term recomputed where the auxiliary law changed, then
recompute_path!(b°, b.WW).  Returns (success, critical) per block.
"""
const _PAR_NAMES = Dict(
    DMT_MODEL_FHN => Dict(:ϵ => 0, :s => 1, :γ => 2, :β => 3, :σ => 4),
    DMT_MODEL_LORENZ => Dict(:s => 0, :r => 1, :β => 2))
function set_proposal_law!(x::DeviceBlocks, θ°::AbstractVector, pnames::AbstractVector; skip=0)
    names = get(_PAR_NAMES, x.se.model, Dict{Symbol,Int}())
    idx = Int32[p isa Symbol ? names[p] : Int32(p) for p in pnames]
    val = Float64.(θ°)
    ok = Vector{UInt8}(undef, x.b1 - x.b0)
    crit = Vector{UInt8}(undef, x.b1 - x.b0)
    check(ccall((:dmt_set_proposal_law, libdmt), Int32,
        (Ptr{Cvoid}, Int32, Int64, Int64, Int32, Ptr{Int32}, Ptr{Float64}, Int32, Ptr{UInt8},
         Ptr{UInt8}), x.se.h, x.layout, x.b0, x.b1, length(idx), idx, val, skip, ok, crit))
    Bool.(ok), Bool.(crit)
end

"find_W_for_X!(b) (src/block.jl:118-131): u.WW from u.XX under the accepted laws."
find_W_for_X!(x::DeviceBlocks) = check(ccall((:dmt_find_W_for_X, libdmt), Int32,
    (Ptr{Cvoid}, Int32, Int64, Int64), x.se.h, x.layout, x.b0, x.b1))

# ---- swaps, histories (src/biblock.jl:135-259)
_swap!(x, what) = check(ccall((:dmt_swap, libdmt), Int32,
    (Ptr{Cvoid}, Int32, Int32, Int64, Int64), x.se.h, x.layout, what, x.b0, x.b1))
swap_paths!(x::DeviceBlocks) = _swap!(x, DMT_SWAP_XX | DMT_SWAP_WW)
swap_XX!(x::DeviceBlocks) = _swap!(x, DMT_SWAP_XX)
swap_WW!(x::DeviceBlocks) = _swap!(x, DMT_SWAP_WW)
swap_PP!(x::DeviceBlocks) = _swap!(x, DMT_SWAP_PP)
swap_ll!(x::DeviceBlocks) = _swap!(x, DMT_SWAP_LL)

save_ll!(x::DeviceBlocks, i::Int) = check(ccall((:dmt_save_ll, libdmt), Int32,
    (Ptr{Cvoid}, Int32, Int64, Int64, Int64), x.se.h, x.layout, x.b0, x.b1, i))

"set_ll!(b, i, v) (src/block.jl:82-86): ll_history[i] of bb.b (unit DMT_U) or bb.b°."
function set_ll!(x::DeviceBlocks, i::Int, v; unit=DMT_U)
    vals = Vector{Float64}(undef, x.b1 - x.b0)
    vals .= v
    check(ccall((:dmt_set_ll, libdmt), Int32,
                (Ptr{Cvoid}, Int32, Int32, Int64, Int64, Int64, Ptr{Float64}),
                x.se.h, x.layout, unit, x.b0, x.b1, i, vals))
end

function set_accepted!(x::DeviceBlocks, i::Int, v)
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
