"""
    MPPIHip

Julia `ccall` binding of libmppi_hip.so (include/mppi.h) that reproduces the reference's Julia controller API:

    mppi_step!(m, d)         src/Humanoid_mppi_v3.jl:154-171, src/cartpole_mppi.jl:103-115
    mppi_controller!(m, d)   src/Humanoid_mppi_v3.jl:173-179  (the `controller=` callback of visualise!)
    mppi_update!(m, d)       src/mppi.jl:83-99

so a reference script switches with

    using MPPIHip
    ctl = MPPIHip.Controller("humanoid_v3"; dynamics = :cross_attention, weights = "ca_humanoid.blob")
    visualise!(model, data; controller = (m, d) -> MPPIHip.mppi_controller!(ctl, m, d))

The humanoid costs read the REAL environment's kinematics on every call (src/Humanoid_mppi_v3.jl:53-99 reads the
global `data`'s cvel / xpos; src/Humanoid_mppi.jl:89-106 its xpos).  Every humanoid solve therefore builds the
per-solve context row from `d` with the reference's own index expressions (`humanoid_v3_context`,
`humanoid_v1_context`, evaluated on MuJoCo.jl's arrays exactly as the reference evaluates them) and passes it
through mppi_solve_ex.  Body ids come from MuJoCo.body(m, name).id on the first call (or `body_ids=` at
construction).

Arrays stay in Julia's column-major layout: U is (nu, H) and injected noise (nu, H, K), passed with
MPPI_FLAG_COLMAJOR. The engine computes in Float32 (Float64 states are converted at the boundary; that
conversion is part of the parity tolerance, DESIGN.md). Untested in this build image (no Julia toolchain).
"""
module MPPIHip

const LIB = get(ENV, "MPPI_HIP_LIB", joinpath(@__DIR__, "..", "lib", "libmppi_hip.so"))

const DYN_CARTPOLE, DYN_MLP, DYN_CROSS_ATTN, DYN_FEATURE_ATTN = Cint(1), Cint(2), Cint(3), Cint(4)
const COST = Dict(:cartpole => Cint(1), :cartpole_est => Cint(2), :humanoid_v3 => Cint(3),
                  :quad_jl => Cint(4), :quad_est => Cint(5), :humanoid_v1 => Cint(6))
const FLAG_SHIFT, FLAG_COLMAJOR, FLAG_U0_BEFORE = Cint(0x1), Cint(0x2), Cint(0x10)
const CTX_MAX = 8

# must match `mppi_io` in include/mppi.h (7 pointers)
struct MPPIIo
    x0::Ptr{Float32}; U::Ptr{Float32}; noise::Ptr{Float32}; costs::Ptr{Float32}
    weights::Ptr{Float32}; u0::Ptr{Float32}; ctx::Ptr{Float32}
end

# must match `mppi_config` in include/mppi.h field for field
mutable struct Config
    nx::Int32; nu::Int32; H::Int32; K::Int32; max_batch::Int32
    lambda::Float32; sigma::Float32; ctrl_clamp::Float32; U_clamp::Float32; norm_eps::Float32
    shift_fill::Float32; terminal_weight::Float32; update_mode::Int32; precision::Int32
    r0::Int32; r1::Int32; r2::Int32; r3::Int32
    Config() = new(0, 0, 0, 0, 0, 0f0, 0f0, 0f0, 0f0, 0f0, 0f0, 0f0, 0, 0, 0, 0, 0, 0)
end

struct MPPIError <: Exception
    code::Cint
    msg::String
end
Base.showerror(io::IO, e::MPPIError) = print(io, "MPPI error ", e.code, ": ", e.msg)

function check(rc::Cint)
    rc == 0 && return rc
    throw(MPPIError(rc, unsafe_string(ccall((:mppi_last_error, LIB), Cstring, ()))))
end

function preset(name::AbstractString; kw...)
    cfg = Config()
    check(ccall((:mppi_preset, LIB), Cint, (Cstring, Ref{Config}), name, cfg))
    for (k, v) in kw
        setfield!(cfg, k, convert(fieldtype(Config, k), v))
    end
    return cfg
end

mutable struct Controller
    handle::Ptr{Cvoid}
    cfg::Config
    preset::String
    U::Matrix{Float32}          # nominal sequence (nu, H): the reference's U_global
    seed::UInt64
    calls::UInt64
    ctx::Vector{Float32}        # per-solve cost context (humanoid real-env terms), CTX_MAX floats
    cost::Symbol
    body_ids::Any               # (shin_left, shin_right, foot_left, foot_right) 0-based MuJoCo ids, or nothing
    u0_before::Bool             # src/quadruped_datacollection.py:170: apply U[:,1] before the update
end

"""
    Controller(preset; dynamics=:cartpole, weights=nothing, cost=nothing, device=0, seed=0, kw...)

`weights` is a weight blob written by mppi_hip.nets.pack_blob (Python) for :mlp / :cross_attention.
"""
function Controller(name::AbstractString; dynamics::Symbol = :cartpole, weights = nothing, cost = nothing,
                    device::Integer = 0, seed::Integer = 0, body_ids = nothing, u0_before::Bool = false, kw...)
    cfg = preset(name; kw...)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:mppi_create, LIB), Cint, (Ref{Config}, Cint, Ref{Ptr{Cvoid}}), cfg, device, h))
    ck = cost === nothing ? (name == "humanoid_v1" ? :humanoid_v1 : startswith(name, "humanoid") ? :humanoid_v3 :
                             startswith(name, "quad") ? :quad_jl : endswith(name, "_est") ? :cartpole_est :
                             :cartpole) : cost
    c = Controller(h[], cfg, String(name), zeros(Float32, cfg.nu, cfg.H), UInt64(seed), 0,
                   zeros(Float32, CTX_MAX), ck, body_ids, u0_before)
    finalizer(c -> ccall((:mppi_destroy, LIB), Cvoid, (Ptr{Cvoid},), c.handle), c)
    if dynamics == :cartpole
        check(ccall((:mppi_load_dynamics, LIB), Cint, (Ptr{Cvoid}, Cint, Ptr{Cvoid}, Csize_t), c.handle,
                    DYN_CARTPOLE, C_NULL, 0))
    else
        blob = read(weights)
        kind = dynamics == :mlp ? DYN_MLP : dynamics == :feature_attention ? DYN_FEATURE_ATTN : DYN_CROSS_ATTN
        check(ccall((:mppi_load_dynamics, LIB), Cint, (Ptr{Cvoid}, Cint, Ptr{UInt8}, Csize_t), c.handle, kind,
                    blob, length(blob)))
    end
    check(ccall((:mppi_set_cost, LIB), Cint, (Ptr{Cvoid}, Cint, Ptr{Float32}, Cint), c.handle, COST[ck],
                C_NULL, 0))
    return c
end

state(d) = Float32.(vcat(vec(d.qpos), vec(d.qvel)))

# src/Humanoid_mppi_v3.jl:22-25, verbatim in meaning: the flat index into MuJoCo.jl's cvel array
get_body_vx(d, body_id) = d.cvel[body_id * 6 - 5 + 3]

"0-based MuJoCo body ids the humanoid costs read, via MuJoCo.body(m, name).id (the reference's own lookups)."
function humanoid_body_ids(m)
    mj = getfield(Main, :MuJoCo)
    bid(n) = Base.invokelatest(mj.body, m, n).id
    return (shin_left = bid("shin_left"), shin_right = bid("shin_right"), foot_left = bid("foot_left"),
            foot_right = bid("foot_right"))
end

"""Context row of MPPI_COST_HUMANOID_V3 from the real environment `d`: src/Humanoid_mppi_v3.jl:53-99 evaluated
as the reference evaluates it (cvel / xpos of the global data), [2, 0, 1.28, swing_foot_x, swing_knee_x, const,
0, 0] with const = -0.15 swing_vx + 2 clr^2 [clr < 0.05] + 0.5 lat^2 [lat < 0] (the terms constant over k, t)."""
function humanoid_v3_context(d, ids)
    if get_body_vx(d, ids.shin_left) > get_body_vx(d, ids.shin_right)
        swing, stance, knee = ids.foot_left, ids.foot_right, ids.shin_left
    else
        swing, stance, knee = ids.foot_right, ids.foot_left, ids.shin_right
    end
    k = -0.15 * get_body_vx(d, swing)                                  # :78-79
    clearance = d.xpos[swing + 1, 3] - d.xpos[stance + 1, 3]           # :86-91
    clearance < 0.05 && (k += 2.0 * abs2(clearance))
    lateral = d.xpos[ids.foot_left + 1, 2] - d.xpos[ids.foot_right + 1, 2]  # :93-99
    lateral < 0 && (k += 0.5 * abs2(lateral))
    return Float32[2.0, 0.0, 1.28, d.xpos[swing + 1, 1], d.xpos[knee + 1, 1], k, 0, 0]
end

"""Context row of MPPI_COST_HUMANOID_V1 (src/Humanoid_mppi.jl:89-106): [2, 0, 1.28, left_foot_x, right_foot_x,
0.01 (right_z - left_z), 0.1 |left_y - right_y|, 0]; the kernel picks the swing side per rollout step t."""
function humanoid_v1_context(d, ids)
    l, r = ids.foot_left + 1, ids.foot_right + 1
    return Float32[2.0, 0.0, 1.28, d.xpos[l, 1], d.xpos[r, 1], 0.01 * (d.xpos[r, 3] - d.xpos[l, 3]),
                   0.1 * abs(d.xpos[l, 2] - d.xpos[r, 2]), 0]
end

function _context!(c::Controller, m, d)
    (c.cost == :humanoid_v3 || c.cost == :humanoid_v1) || return C_NULL
    c.body_ids === nothing && (c.body_ids = humanoid_body_ids(m))
    c.ctx .= c.cost == :humanoid_v3 ? humanoid_v3_context(d, c.body_ids) : humanoid_v1_context(d, c.body_ids)
    return pointer(c.ctx)
end

function _solve!(c::Controller, m, d; flags::Cint = Cint(0), noise = nothing)
    x0 = state(d)
    u0 = zeros(Float32, c.cfg.nu)
    c.calls += 1
    seed = xor(c.seed << 32, c.calls)
    nz = noise === nothing ? Float32[] : Float32.(noise)   # (nu, H, K) column-major, already scaled
    GC.@preserve x0 u0 nz c begin
        io = MPPIIo(pointer(x0), pointer(c.U), noise === nothing ? C_NULL : pointer(nz), C_NULL, C_NULL,
                    pointer(u0), _context!(c, m, d))
        check(ccall((:mppi_solve_ex, LIB), Cint, (Ptr{Cvoid}, Cint, Ref{MPPIIo}, UInt64, Cint),
                    c.handle, 1, io, seed, flags | FLAG_COLMAJOR))
    end
    return u0
end

"mppi_step!: noise -> rollout -> softmin -> U update (no shift); U_global kept in `c.U`."
mppi_step!(c::Controller, m, d; noise = nothing) = (_solve!(c, m, d; noise = noise); nothing)

"mppi_controller!: mppi_step!, then d.ctrl .= U[:,1] and the receding-horizon shift (0.1 decay or zero fill)."
function mppi_controller!(c::Controller, m, d; noise = nothing)
    flags = FLAG_SHIFT | (c.u0_before ? FLAG_U0_BEFORE : Cint(0))
    u0 = _solve!(c, m, d; flags = flags, noise = noise)
    d.ctrl .= u0
    return nothing
end

mppi_update!(c::Controller, m, d; kw...) = mppi_controller!(c, m, d; kw...)

"x3_layer1: (products, probe error) of the split CA's layer 1 (mppi_x3_layer1; ABI 3)."
function x3_layer1(c::Controller)
    prod = Ref{Cint}(0)
    err = Ref{Cfloat}(0)
    check(ccall((:mppi_x3_layer1, LIB), Cint, (Ptr{Cvoid}, Ref{Cint}, Ref{Cfloat}), c.handle, prod, err))
    return (Int(prod[]), Float32(err[]))
end

"rollout_kernel: the kernel the last solve was routed to (mppi_rollout_kernel; ABI 3)."
rollout_kernel(c::Controller) = unsafe_string(ccall((:mppi_rollout_kernel, LIB), Cstring, (Ptr{Cvoid},), c.handle))

"x3_f16: (form, probe error) of the split CA's fp16 form (mppi_x3_f16; ABI 4): 2 / 1 = on with a one- / two-product last layer, 0 = off."
function x3_f16(c::Controller)
    on = Ref{Cint}(0)
    err = Ref{Cfloat}(0)
    check(ccall((:mppi_x3_f16, LIB), Cint, (Ptr{Cvoid}, Ref{Cint}, Ref{Cfloat}), c.handle, on, err))
    return (Int(on[]), Float32(err[]))
end

end # module
