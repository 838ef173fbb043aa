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

Arrays stay in Julia's column-major layout: U is (nu, H) and injected noise (nu, H, K), passed with
MPPI_FLAG_COLMAJOR. The engine computes in Float32 (Float64 states are converted at the boundary; that
conversion is part of the parity tolerance, DESIGN.md). Untested in this build image (no Julia toolchain).
"""
module MPPIHip

const LIB = get(ENV, "MPPI_HIP_LIB", joinpath(@__DIR__, "..", "lib", "libmppi_hip.so"))

const DYN_CARTPOLE, DYN_MLP, DYN_CROSS_ATTN, DYN_FEATURE_ATTN = Cint(1), Cint(2), Cint(3), Cint(4)
const COST = Dict(:cartpole => Cint(1), :cartpole_est => Cint(2), :humanoid_v3 => Cint(3),
                  :quad_jl => Cint(4), :quad_est => Cint(5))
const FLAG_SHIFT, FLAG_COLMAJOR, FLAG_U0_BEFORE = Cint(0x1), Cint(0x2), Cint(0x10)
const CTX_MAX = 8

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
end

"""
    Controller(preset; dynamics=:cartpole, weights=nothing, cost=nothing, device=0, seed=0, kw...)

`weights` is a weight blob written by mppi_hip.nets.pack_blob (Python) for :mlp / :cross_attention.
"""
function Controller(name::AbstractString; dynamics::Symbol = :cartpole, weights = nothing, cost = nothing,
                    device::Integer = 0, seed::Integer = 0, kw...)
    cfg = preset(name; kw...)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:mppi_create, LIB), Cint, (Ref{Config}, Cint, Ref{Ptr{Cvoid}}), cfg, device, h))
    c = Controller(h[], cfg, String(name), zeros(Float32, cfg.nu, cfg.H), UInt64(seed), 0,
                   zeros(Float32, CTX_MAX))
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
    ck = cost === nothing ? (startswith(name, "humanoid") ? :humanoid_v3 : startswith(name, "quad") ?
                             :quad_jl : endswith(name, "_est") ? :cartpole_est : :cartpole) : cost
    check(ccall((:mppi_set_cost, LIB), Cint, (Ptr{Cvoid}, Cint, Ptr{Float32}, Cint), c.handle, COST[ck],
                C_NULL, 0))
    return c
end

state(d) = Float32.(vcat(vec(d.qpos), vec(d.qvel)))

function _solve!(c::Controller, d; flags::Cint = Cint(0), noise = nothing)
    x0 = state(d)
    u0 = zeros(Float32, c.cfg.nu)
    c.calls += 1
    seed = xor(c.seed << 32, c.calls)
    nz = noise === nothing ? C_NULL : Float32.(noise)   # (nu, H, K) column-major, already scaled
    check(ccall((:mppi_solve, LIB), Cint,
                (Ptr{Cvoid}, Cint, Ptr{Float32}, Ptr{Float32}, Ptr{Float32}, UInt64, Ptr{Float32}, Ptr{Float32}, Cint),
                c.handle, 1, x0, c.U, nz, seed, C_NULL, u0, flags | FLAG_COLMAJOR))
    return u0
end

"mppi_step!: noise -> rollout -> softmin -> U update (no shift); U_global kept in `c.U`."
mppi_step!(c::Controller, m, d; noise = nothing) = (_solve!(c, d; noise = noise); nothing)

"mppi_controller!: mppi_step!, then d.ctrl .= U[:,1] and the receding-horizon shift (0.1 decay or zero fill)."
function mppi_controller!(c::Controller, m, d; noise = nothing)
    flags = FLAG_SHIFT | (c.preset == "quad_collect_py" ? FLAG_U0_BEFORE : Cint(0))
    u0 = _solve!(c, d; flags = flags, noise = noise)
    d.ctrl .= u0
    return nothing
end

mppi_update!(c::Controller, m, d; kw...) = mppi_controller!(c, m, d; kw...)

end # module
