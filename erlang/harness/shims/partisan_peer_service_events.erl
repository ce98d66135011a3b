%% partisan_peer_service_events shim of the parity harness: notify/1 of the
%% HyParView manager (hv:1598-1599) reaches the running node's Plumtree
%% state at once, as the gen_event callback -> plumtree update/1 -> decode ->
%% handle_cast({update, Members}) chain does (events:66-67, pt:181-183,
%% :314-336).  Nothing in the HyParView phase reads Plumtree state, so this
%% equals the round model's replay of the notifies before the Plumtree phase.
-module(partisan_peer_service_events).
-export([update/1]).

update(Active) ->
    Names = [Name || #{name := Name} <- sets:to_list(Active)],
    psim_harness:pt_update(Names),
    ok.
