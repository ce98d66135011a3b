%% partisan_gpu_sim_fault_model -- the omission commands of partisan's crash
%% fault model (test/prop_partisan_crash_fault_model.erl:93-229) over the
%% simulator, for a pluggable-manager handle.
%%
%% In the reference each command installs or removes an interposition fun in
%% one node's pluggable manager (add_interposition_fun/2,
%% remove_interposition_fun/1, pluggable:297-326); the manager folds the funs
%% over every forwarded (:669-684) and received (:634-646) message and drops
%% the ones that come out `undefined`.  Here the same funs are named by their
%% (source, destination) pair and applied on the GPU to every strategy
%% message of the next rounds; a dropped send never reaches the connection
%% lookup or the dispatch draw (pluggable:727-760), exactly as there.
%% Nodes are simulator ids; Name-based callers map 'n<id>@sim' to the id.
-module(partisan_gpu_sim_fault_model).
-export([crash/2, begin_omission/2, end_omission/2,
         begin_receive_omission/3, end_receive_omission/3,
         begin_send_omission/3, end_send_omission/3,
         resolve_all_faults_with_heal/1, resolve_all_faults_with_crash/2]).

%% crash/2 (:82-91): crash-stop with asynchronous failure detection
crash(Sim, Node) -> partisan_gpu_sim:crash(Sim, [Node]).

%% begin_omission/1, end_omission/1 (:93-114): the `faulted` flag read by the
%% trace orchestrator's interposition funs (partisan_trace_orchestrator:621-656):
%% every strategy message the node sends or receives is dropped
begin_omission(Sim, Node) -> partisan_gpu_sim:begin_omission(Sim, [Node]).
end_omission(Sim, Node) -> partisan_gpu_sim:end_omission(Sim, [Node]).

%% begin_receive_omission/2 (:117-140): {receive_omission, Source} at
%% Destination drops what Destination receives from Source
begin_receive_omission(Sim, Source, Destination) ->
    partisan_gpu_sim:begin_receive_omission(Sim, [Source], [Destination]).
end_receive_omission(Sim, Source, Destination) ->
    partisan_gpu_sim:end_receive_omission(Sim, [Source], [Destination]).

%% begin_send_omission/2 (:158-181): {send_omission, Destination} at Source
%% drops what Source forwards to Destination
begin_send_omission(Sim, Source, Destination) ->
    partisan_gpu_sim:begin_send_omission(Sim, [Source], [Destination]).
end_send_omission(Sim, Source, Destination) ->
    partisan_gpu_sim:end_send_omission(Sim, [Source], [Destination]).

%% resolve_all_faults_with_heal/0 (:198-229): every interposition fun removed
resolve_all_faults_with_heal(Sim) -> partisan_gpu_sim:clear_faults(Sim).

%% resolve_all_faults_with_crash/0 (:231-290): the nodes that hold an
%% interposition fun are crashed instead, then every fun is removed.
%% Faulted is the list of those nodes (the caller's record of its commands:
%% the simulator does not list installed funs).
resolve_all_faults_with_crash(Sim, Faulted) ->
    case partisan_gpu_sim:crash(Sim, lists:usort(Faulted)) of
        ok -> partisan_gpu_sim:clear_faults(Sim);
        Error -> Error
    end.
