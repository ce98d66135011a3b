%% partisan_gpu_sim_peer_service_manager -- the partisan_peer_service_manager
%% behaviour (src/partisan_peer_service_manager.erl:30-67) backed by the MI355X
%% simulator: the whole overlay lives on the GPU, and this gen_server answers
%% for one simulated node (`sim_node` in partisan_config) while the host
%% drives rounds with step/1.  Node names map to ids as 'n<id>@sim'.
%%
%% What each callback does here, against the HyParView manager it replaces
%% (hv = src/partisan_hyparview_peer_service_manager.erl):
%%   members/0, get_local_state/0   the simulated node's active view (hv:261-281)
%%   join/1                         the node starts and sends JOIN to the contact
%%                                  in the next round (hv:500-515); a node that
%%                                  already runs cannot join again
%%   sync_join/1                    join/1, then rounds until the contact is in the
%%                                  active view (hv: {error, not_implemented}, :229-230)
%%   leave/0,1                      error, as hv:233-238 (SURVEY App. A Q13)
%%   update_members/1               {error, not_implemented}, as hv:139-140
%%   on_up/2, on_down/2             functions fired when the named node enters /
%%                                  leaves the active view, checked after every
%%                                  step (the pluggable manager's semantics,
%%                                  pluggable:136-145, :1365-1388; hv answers
%%                                  not_implemented, :131-136)
%%   inject_partition/2             the nodes within TTL hops of Origin over active
%%                                  views are cut off from the rest (a network
%%                                  partition, DESIGN.md section 2; hv:244-246,
%%                                  :1731-1769 floods the same TTL)
%%                                  one partition at a time per simulator handle:
%%                                  a second injection before the first is
%%                                  resolved answers {error, already_partitioned}
%%                                  (managers sharing a handle through sim_handle
%%                                  share that one cut)
%%   resolve_partition/1, partitions/0   hv:249-255, :1771-1797
%%   send_message/2, forward_message/2..5, cast_message/3..5, receive_message/2
%%                                  application traffic is not simulated (only
%%                                  membership and broadcast are):
%%                                  {error, not_implemented}
%%   reserve/1                      {error, no_available_slots} (no reservations
%%                                  are modelled, DESIGN.md section 2)
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
-export([step/1, broadcast/1, start_seed/0, sim/0]).
-export([init/1, handle_call/3, handle_cast/2, handle_info/2, terminate/2, code_change/3]).

-define(NONE, 16#FFFFFFFF).

-record(state, {sim,
                me :: non_neg_integer(),
                n :: pos_integer(),
                started = false :: boolean(),
                msg = 0 :: non_neg_integer(),
                active = [] :: [non_neg_integer()],      % the active view after the last step
                up_funs = #{} :: #{atom() => [fun(() -> any())]},
                down_funs = #{} :: #{atom() => [fun(() -> any())]},
                partition = undefined :: undefined | {reference(), [non_neg_integer()]}}).

start_link() -> gen_server:start_link({local, ?MODULE}, ?MODULE, [], []).

members() -> gen_server:call(?MODULE, members, infinity).
members_for_orchestration() -> members().
myself() -> partisan_peer_service_manager:myself().
get_local_state() -> gen_server:call(?MODULE, get_local_state, infinity).
join(#{name := Name}) -> gen_server:call(?MODULE, {join, id(Name)}, infinity).
sync_join(#{name := Name}) -> gen_server:call(?MODULE, {sync_join, id(Name)}, infinity).
leave() -> error.                       % hv:233-238: leave is not implemented
leave(_) -> error.
update_members(_) -> {error, not_implemented}.
on_down(#{name := Name}, Fun) -> on_down(Name, Fun);
on_down(Name, Fun) when is_atom(Name) -> gen_server:call(?MODULE, {on_down, Name, Fun}, infinity).
on_up(#{name := Name}, Fun) -> on_up(Name, Fun);
on_up(Name, Fun) when is_atom(Name) -> gen_server:call(?MODULE, {on_up, Name, Fun}, infinity).
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
partitions() -> gen_server:call(?MODULE, partitions, infinity).
inject_partition(#{name := Origin}, TTL) -> inject_partition(Origin, TTL);
inject_partition(Origin, TTL) when is_atom(Origin), is_integer(TTL), TTL >= 0 ->
    gen_server:call(?MODULE, {inject_partition, id(Origin), TTL}, infinity).
resolve_partition(Ref) -> gen_server:call(?MODULE, {resolve_partition, Ref}, infinity).

%% host controls: advance the simulation, originate a Plumtree broadcast at
%% a node, start this node as a seed (no contact), the simulator handle
step(Rounds) -> gen_server:call(?MODULE, {step, Rounds}, infinity).
broadcast(Root) -> gen_server:call(?MODULE, {broadcast, Root}, infinity).
start_seed() -> gen_server:call(?MODULE, start_seed, infinity).
sim() -> gen_server:call(?MODULE, sim, infinity).

init([]) ->
    N = partisan_config:get(sim_nodes, 32),
    Me = partisan_config:get(sim_node, 0),
    Cfg = #{n_nodes => N, seed => partisan_config:get(sim_seed, 1),
            max_active_size => partisan_config:get(max_active_size, 6),
            min_active_size => partisan_config:get(min_active_size, 3),
            max_passive_size => partisan_config:get(max_passive_size, 30),
            arwl => partisan_config:get(arwl, 5), prwl => partisan_config:get(prwl, 30),
            %% sim_xbot = true: partisan_hyparview_xbot_peer_service_manager's
            %% semantics (optimization rounds every xbot_period rounds)
            manager => case partisan_config:get(sim_xbot, false) of true -> 2; _ -> 0 end,
            xbot_period => partisan_config:get(sim_xbot_period, 35)},
    {ok, Sim} = case partisan_config:get(sim_handle, undefined) of
                    undefined ->
                        {ok, H0} = partisan_gpu_sim:create(Cfg),
                        %% views in this VM's sets v1 order (SURVEY App. A Q1):
                        %% erlang:phash/2 of every simulated node_spec
                        ok = partisan_gpu_sim:set_phash_table(H0, partisan_gpu_sim:phash_table(N, fun spec/1)),
                        {ok, H0};
                    H -> {ok, H}
                end,
    %% the node starts at join/1 (or start_seed/0): one start per node
    {ok, #state{sim = Sim, me = Me, n = N}}.

handle_call(members, _From, S) ->
    {reply, {ok, [name(I) || I <- view(S)]}, S};
handle_call(get_local_state, _From, S) ->
    {reply, {ok, {state, view(S), 1}}, S};
handle_call({join, Id}, _From, S) ->
    {Reply, S1} = start(Id, S),
    {reply, Reply, S1};
handle_call({sync_join, Id}, _From, S) ->
    case start(Id, S) of
        {ok, S1} ->
            Rounds = partisan_config:get(sim_sync_join_rounds, 20),
            {Reply, S2} = step_until(fun(St) -> lists:member(Id, St#state.active) end, Rounds, S1),
            {reply, Reply, S2};
        {Error, S1} ->
            {reply, Error, S1}
    end;
handle_call(start_seed, _From, S) ->
    {Reply, S1} = start(?NONE, S),
    {reply, Reply, S1};
handle_call({on_up, Name, Fun}, _From, S = #state{up_funs = U}) ->
    {reply, ok, S#state{up_funs = maps:update_with(Name, fun(L) -> L ++ [Fun] end, [Fun], U)}};
handle_call({on_down, Name, Fun}, _From, S = #state{down_funs = D}) ->
    {reply, ok, S#state{down_funs = maps:update_with(Name, fun(L) -> L ++ [Fun] end, [Fun], D)}};
handle_call({step, Rounds}, _From, S) ->
    {Reply, S1} = do_step(Rounds, S),
    {reply, Reply, S1};
handle_call({broadcast, Root}, _From, S = #state{sim = Sim, msg = M}) ->
    {reply, partisan_gpu_sim:broadcast(Sim, id(Root), M band 16#FFFF), S#state{msg = M + 1}};
handle_call(partitions, _From, S = #state{partition = undefined}) ->
    {reply, {ok, []}, S};
handle_call(partitions, _From, S = #state{partition = {Ref, Cut}}) ->
    %% the active peers of this node on the other side of the cut (hv:1763-1765)
    Mine = lists:member(S#state.me, Cut),
    Peers = [{Ref, name(P)} || P <- view(S), P =/= S#state.me, lists:member(P, Cut) =/= Mine],
    {reply, {ok, Peers}, S};
handle_call({inject_partition, _, _}, _From, S = #state{partition = {_, _}}) ->
    %% one partition per handle: the network keeps a single cut, so a second
    %% injection would silently replace the first (the reference accumulates
    %% {Ref, Peer} entries per injection, hv:1766-1770)
    {reply, {error, already_partitioned}, S};
handle_call({inject_partition, Origin, TTL}, _From, S = #state{sim = Sim, n = N}) ->
    %% the flood of hv:1731-1769 reaches the nodes within TTL hops of Origin
    %% over active views; they form one side of a network partition
    Cut = flood([Origin], [Origin], TTL, Sim),
    Groups = [case lists:member(I, Cut) of true -> 1; false -> 0 end || I <- lists:seq(0, N - 1)],
    case partisan_gpu_sim:set_partition(Sim, Groups) of
        ok ->
            Ref = make_ref(),
            {reply, {ok, Ref}, S#state{partition = {Ref, Cut}}};
        Error ->
            {reply, Error, S}
    end;
handle_call({resolve_partition, Ref}, _From, S = #state{partition = {Ref, _}, sim = Sim}) ->
    {reply, partisan_gpu_sim:clear_partition(Sim), S#state{partition = undefined}};
handle_call({resolve_partition, _}, _From, S) ->
    {reply, ok, S};                         % an unknown reference changes nothing (hv:1777-1790)
handle_call(sim, _From, S = #state{sim = Sim}) ->
    {reply, {ok, Sim}, S};
handle_call(_, _From, S) -> {reply, {error, not_implemented}, S}.

handle_cast(_, S) -> {noreply, S}.
handle_info(_, S) -> {noreply, S}.
terminate(_, _) -> ok.
code_change(_, S, _) -> {ok, S}.

%% ------------------------------------------------------------ internal
start(_Contact, S = #state{started = true}) ->
    {{error, already_started}, S};
start(Contact, S = #state{sim = Sim, me = Me}) ->
    case partisan_gpu_sim:join(Sim, [Me], [Contact]) of
        ok -> {ok, S#state{started = true}};
        Error -> {Error, S}
    end.

view(#state{sim = Sim, me = Me}) ->
    {ok, Ids} = partisan_gpu_sim:active(Sim, Me),
    Ids.

do_step(Rounds, S = #state{sim = Sim}) ->
    case partisan_gpu_sim:step(Sim, Rounds) of
        {ok, Stats} -> {{ok, Stats}, fire(S)};
        Error -> {Error, S}
    end.

step_until(_Done, 0, S) ->
    {{error, timeout}, S};
step_until(Done, Left, S) ->
    case do_step(1, S) of
        {{ok, _}, S1} ->
            case Done(S1) of
                true -> {ok, S1};
                false -> step_until(Done, Left - 1, S1)
            end;
        {Error, S1} ->
            {Error, S1}
    end.

%% on_up / on_down functions of the peers that entered / left the active view
fire(S = #state{active = Old, up_funs = U, down_funs = D, me = Me}) ->
    New = view(S),
    [[F() || F <- maps:get(name(P), U, [])] || P <- New -- Old, P =/= Me],
    [[F() || F <- maps:get(name(P), D, [])] || P <- Old -- New, P =/= Me],
    S#state{active = New}.

%% breadth-first over active views, TTL hops out from the frontier
flood(Seen, _Frontier, 0, _Sim) -> lists:usort(Seen);
flood(Seen, [], _TTL, _Sim) -> lists:usort(Seen);
flood(Seen, Frontier, TTL, Sim) ->
    Next = lists:usort(lists:append([begin {ok, A} = partisan_gpu_sim:active(Sim, F), A end
                                     || F <- Frontier])) -- Seen,
    flood(Seen ++ Next, Next, TTL - 1, Sim).

name(Id) -> list_to_atom(lists:flatten(io_lib:format("n~10..0B@sim", [Id]))).
%% the node_spec of simulated node Id (the harness's, DESIGN.md section 2)
spec(Id) ->
    #{name => name(Id),
      listen_addrs => [#{ip => partisan_gpu_sim:spec_ip(Id), port => 9090}],
      channels => [undefined], parallelism => 1}.
id(Name) when is_atom(Name) ->
    [$n | Rest] = atom_to_list(Name),
    list_to_integer(lists:takewhile(fun(C) -> C >= $0 andalso C =< $9 end, Rest));
id(#{name := Name}) -> id(Name);
id(Id) when is_integer(Id) -> Id.
