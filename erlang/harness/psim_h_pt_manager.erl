%% The peer-service manager Plumtree's send/3 calls in the parity harness
%% (partisan_config partisan_peer_service_manager, pt:633-638): cast_message
%% succeeds only over an existing connection of the node's HyParView manager
%% -- the target is in its active view, running, same partition -- and
%% draws nothing (the broadcast process is unseeded, SURVEY App. A Q9).
-module(psim_h_pt_manager).
-export([cast_message/3, myself/0]).

cast_message(Peer, _ServerRef, Msg) ->
    Src = get(psim_h_node),
    Name = case Peer of #{name := N} -> N; N when is_atom(N) -> N end,
    Kind = case Peer of #{} -> map; _ -> atom end,       % the identity quirk, App. A Q6
    psim_harness:pt_send(Src, Name, Kind, Msg).

myself() -> partisan_peer_service_manager:myself().
