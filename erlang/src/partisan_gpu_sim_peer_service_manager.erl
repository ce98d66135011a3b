%% partisan_gpu_sim_peer_service_manager -- the partisan_peer_service_manager
%% behaviour (src/partisan_peer_service_manager.erl:30-67) backed by the MI355X
%% simulator: the whole overlay lives on the GPU, and this gen_server answers
%% for one simulated node (`sim_node` in partisan_config) while the host
%% drives rounds with step/1.  Node names map to ids as 'n<id>@sim'.
-module(partisan_gpu_sim_peer_service_manager).
-behaviour(gen_server).
-behaviour(partisan_peer_service_manager).

-export([start_link/0, members/0, members_for_orchestration/0, myself/0,
         get_local_state/0, join/1, sync_join/1, leave/0, leave/1,
         update_members/1, on_down/2, on_up/2, send_message/2,
         forward_message/2, cast_message/3, forward_message/3,
         cast_message/4, forward_message/4, cast_message/5,
         forward_message/5, receive_message/2, decode/1, reserve/1,
         partitions/0, inject_partition/2, resolve_partition/1]).
-export([step/1, broadcast/1]).
-export([init/1, handle_call/3, handle_cast/2, handle_info/2, terminate/2, code_change/3]).

-record(state, {sim, me :: non_neg_integer(), n :: pos_integer(), msg = 0}).

start_link() -> gen_server:start_link({local, ?MODULE}, ?MODULE, [], []).

members() -> gen_server:call(?MODULE, members, infinity).
members_for_orchestration() -> members().
myself() -> partisan_peer_service_manager:myself().
get_local_state() -> gen_server:call(?MODULE, get_local_state, infinity).
join(#{name := Name}) -> gen_server:call(?MODULE, {join, id(Name)}, infinity).
sync_join(_) -> {error, not_implemented}.
leave() -> error.                       % hv:363-364: leave is not implemented
leave(_) -> error.
update_members(_) -> {error, not_implemented}.
on_down(_, _) -> {error, not_implemented}.
on_up(_, _) -> {error, not_implemented}.
%% application traffic is not simulated: only membership and broadcast are
send_message(_, _) -> {error, not_implemented}.
forward_message(_, _) -> {error, not_implemented}.
cast_message(_, _, _) -> {error, not_implemented}.
forward_message(_, _, _) -> {error, not_implemented}.
cast_message(_, _, _, _) -> {error, not_implemented}.
forward_message(_, _, _, _) -> {error, not_implemented}.
cast_message(_, _, _, _, _) -> {error, not_implemented}.
forward_message(_, _, _, _, _) -> {error, not_implemented}.
receive_message(_, _) -> {error, not_implemented}.
decode(Active) -> Active.
reserve(_) -> {error, no_available_slots}.
partitions() -> {ok, []}.
inject_partition(_, _) -> {error, not_implemented}.
resolve_partition(_) -> {error, not_implemented}.

%% host controls: advance the simulation, originate a Plumtree broadcast
step(Rounds) -> gen_server:call(?MODULE, {step, Rounds}, infinity).
broadcast(Root) -> gen_server:call(?MODULE, {broadcast, Root}, infinity).

init([]) ->
    N = partisan_config:get(sim_nodes, 32),
    Me = partisan_config:get(sim_node, 0),
    Cfg = #{n_nodes => N, seed => partisan_config:get(sim_seed, 1),
            max_active_size => partisan_config:get(max_active_size, 6),
            min_active_size => partisan_config:get(min_active_size, 3),
            max_passive_size => partisan_config:get(max_passive_size, 30),
            arwl => partisan_config:get(arwl, 5), prwl => partisan_config:get(prwl, 30)},
    {ok, Sim} = partisan_gpu_sim:create(Cfg),
    ok = partisan_gpu_sim:join(Sim, [Me], [16#FFFFFFFF]),
    {ok, #state{sim = Sim, me = Me, n = N}}.

handle_call(members, _From, S = #state{sim = Sim, me = Me}) ->
    {ok, Ids} = partisan_gpu_sim:active(Sim, Me),
    {reply, {ok, [name(I) || I <- Ids]}, S};
handle_call(get_local_state, _From, S = #state{sim = Sim, me = Me}) ->
    {ok, Ids} = partisan_gpu_sim:active(Sim, Me),
    {reply, {ok, {state, Ids, 1}}, S};
handle_call({join, Id}, _From, S = #state{sim = Sim, me = Me}) ->
    {reply, partisan_gpu_sim:join(Sim, [Id], [Me]), S};
handle_call({step, Rounds}, _From, S = #state{sim = Sim}) ->
    {reply, partisan_gpu_sim:step(Sim, Rounds), S};
handle_call({broadcast, Root}, _From, S = #state{sim = Sim, msg = M}) ->
    {reply, partisan_gpu_sim:broadcast(Sim, Root, M band 16#FFFF), S#state{msg = M + 1}};
handle_call(_, _From, S) -> {reply, {error, not_implemented}, S}.

handle_cast(_, S) -> {noreply, S}.
handle_info(_, S) -> {noreply, S}.
terminate(_, _) -> ok.
code_change(_, S, _) -> {ok, S}.

name(Id) -> list_to_atom(lists:flatten(io_lib:format("n~10..0B@sim", [Id]))).
id(Name) ->
    [$n | Rest] = atom_to_list(Name),
    list_to_integer(lists:takewhile(fun(C) -> C >= $0 andalso C =< $9 end, Rest)).
