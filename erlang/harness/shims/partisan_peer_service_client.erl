%% partisan_peer_service_client shim of the parity harness: a "connection"
%% is a recording proxy process.  start_link succeeds iff the target node is
%% running and in the caller's partition group -- the round model's
%% connect rule (DESIGN.md section 2); a send through the proxy is logged
%% as an emitted record of the current round (src, seq) and answered ok.
%% The proxy is linked to the caller, as the real client (client:51-80).
-module(partisan_peer_service_client).
-export([start_link/4]).

start_link(#{name := Name}, _ListenAddr, _Channel, From) ->
    Src = get(psim_h_node),
    Dst = psim_harness:id_of(Name),
    case psim_harness:reachable(Src, Dst) of
        true ->
            Pid = spawn(fun() -> proxy(Src, Dst) end),
            link(Pid),
            _ = From,
            psim_harness:register_conn(Src, Dst, Pid),
            {ok, Pid};
        false ->
            {error, normal}
    end.

proxy(Src, Dst) ->
    receive
        {'$gen_call', From, {send_message, Msg}} ->
            psim_harness:record(Src, Dst, Msg),
            gen_server:reply(From, ok),
            proxy(Src, Dst);
        stop ->
            ok
    end.
